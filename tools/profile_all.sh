#!/bin/bash
# Every config's rocprofv3 kernel trace + PMC passes (tools/profile.sh), one name per config:
#   c2 headline, c2r8 (rank 0 of the 8-way split), c3 book 1, c4 Cornell volume, c5 book 2.
# Stops at the first failure. Then on the CPU: tools/roofline_report.py <tag> <name> per name.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
B1="--scene final_render_book_1.json --width 1920 --height 1080 --spp 500"
VOL="--scene cornell_box_volume.json --spp 4000"
B2="--scene book2_final_scene_10000_samples.json --width 800 --height 800 --spp 10000"
bash $R/tools/profile.sh c2 --steps 2 || exit 1
bash $R/tools/profile.sh c2r8 --steps 2 --emulate-world 8 --emulate-rank 0 || exit 1
bash $R/tools/profile.sh c3 $B1 --steps 1 || exit 1
bash $R/tools/profile.sh c4 $VOL --steps 1 --warmup 0 || exit 1
TRACE_TIMEOUT=400 PMC_TIMEOUT=200 bash $R/tools/profile.sh c5 $B2 --steps 1 --warmup 0 || exit 1
