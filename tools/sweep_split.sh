#!/bin/bash
# Work-split / batch sweep for the row band of one rank of an N-way split (bench.py --emulate-world),
# the shapes the driver's 2/4/8-GPU runs give each GPU. Lines go to gpurun_out/sweep.jsonl.
NO_TESTS=1 STEPS=5 exec bash "$(dirname "$0")/sweep.sh" \
  "--emulate-world 8 --work-split 16" "--emulate-world 8 --work-split 32" "--emulate-world 8" \
  "--emulate-world 8 --work-split 128" "--emulate-world 8 --work-split 256" \
  "--emulate-world 8 --batch-max 16" "--emulate-world 8 --batch-max 32" \
  "--emulate-world 4" "--emulate-world 4 --work-split 32" \
  "--emulate-world 2" "--emulate-world 2 --work-split 32"
