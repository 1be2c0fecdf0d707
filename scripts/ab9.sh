set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_all.log 2>&1 || { tail -30 gpurun_out/pytest_all.log; exit 1; }
tail -1 gpurun_out/pytest_all.log
timeout -k 10 300 python scripts/sweep_seq.py > gpurun_out/sweep_seq.jsonl 2>/dev/null || exit $?
cat gpurun_out/sweep_seq.jsonl
