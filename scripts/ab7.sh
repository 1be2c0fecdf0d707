set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_all.log 2>&1 || { tail -30 gpurun_out/pytest_all.log; exit 1; }
tail -1 gpurun_out/pytest_all.log
KERNELS="2 0 1" timeout -k 10 600 bash scripts/r1_variants.sh || exit $?
bash scripts/ab6.sh
