#!/bin/bash
# rocprofv3 kernel trace of the VQ microbenchmark (per-kernel durations)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/vqprof
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/vqprof -o vq --output-format csv -- python3 tools/vq_bench.py 20 > gpurun_out/vqprof/run.log 2>&1
echo "rc=$?"
find gpurun_out/vqprof -name "*kernel_stats.csv" | head -3
