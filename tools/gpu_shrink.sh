#!/bin/bash
# generate_batch stepping only the busy slot range: the C3 share twice per process (graph capture vs steady state)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/shrink2.jsonl
for o in '{"batch_shrink": false}' '{"batch_shrink": true}'; do
  C3_REPS=2 timeout -k 10 300 python -u tools/bench_c3.py "$o" >> gpurun_out/shrink2.jsonl 2>> gpurun_out/shrink.err || exit 4
done
