# Build the GEMM lab binaries (one per lab mode) for gfx950, in parallel.
cd "$(dirname "$0")"
for m in 0 1 2 3; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=fast -I ../../include -DVQX_LAB_MODE=$m gemm_lab.hip -o gemm_lab_m$m &
done
for e in 1 2 3; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=fast -I ../../include -DVQX_LAB_EPI=$e gemm_lab.hip -o gemm_lab_e$e &
done
wait
ls -la gemm_lab_m* gemm_lab_e*
