#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/placement_ab.py > gpurun_out/placement_ab.jsonl 2> gpurun_out/placement_ab.err
rc=$?; cat gpurun_out/placement_ab.jsonl; tail -3 gpurun_out/placement_ab.err; exit $rc
