#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/graph_var.jsonl
timeout -k 10 200 python -u tools/graph_var.py default >> gpurun_out/graph_var.jsonl 2>> gpurun_out/graph_var.err || exit $?
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 python -u tools/graph_var.py dev_kernarg >> gpurun_out/graph_var.jsonl 2>> gpurun_out/graph_var.err || exit $?
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 200 python -u tools/graph_var.py no_packet_capture >> gpurun_out/graph_var.jsonl 2>> gpurun_out/graph_var.err || exit $?
cat gpurun_out/graph_var.jsonl
