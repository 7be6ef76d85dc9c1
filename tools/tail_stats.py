import sys, os, json
sys.path.insert(0,'/root/repo')
import torch
import raytrace2_amd as R
for world, t in [(1,8),(8,8),(1,32)]:
    sc=R.Scene('scenes/cornell_box_original.json', R.DEFAULT_SEED)
    tr=R.RayTracer(sc,0); tr.SetSamplesPerPixel(1000); tr.OnResize((1024,1024))
    if world>1: tr.set_partition(2,0,world)
    tr.set_tail_compaction(t)
    tr.Render(1000); tr.synchronize(); tr.Reset(); tr.reset_stats(); tr.Render(1000)
    st=tr.stats(); d=st['diag']
    print(json.dumps({"world":world,"tail":t,"kernel_ms":round(st['kernel_ms'],2),"migrated":st['migrated'],"resumed":st['resumed'],"resumed_drain":d[5],"tries":d[6],"seen":d[7]}))
    tr.close()
