# round-4 lab: 256x256 8-wave pipelined conv GEMM vs conv_gemm_kernel (tools/lab/g8_lab.hip)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/g8
timeout -k 10 120 tools/lab/g8_lab.bin 2>&1 | tee gpurun_out/g8/g8_lab.txt
