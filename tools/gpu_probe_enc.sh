#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
PROBE_TRACE=1 timeout -k 10 300 python tools/enc_bwd_probe.py > gpurun_out/enc_trace.txt 2>&1
