# round-4: codebook widths 64 / 256 -- VQ kernel tests, golden steps, GPU suite, bench (VQ line)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4s; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_step.py -m gpu -x -q -k "vq or golden" --timeout 300 --timeout-method thread > $O/tests_vq.log 2>&1
rc=$?; echo "vq tests rc=$rc"; tail -3 $O/tests_vq.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --fp32-steps 0 --steps 40 > $O/bench.json 2> $O/bench.err || exit $?
python3 -c "
import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['vq'])"
