mkdir -p gpurun_out/r3e2
for nb in 8 32; do for v in f0 f1 f0s f0n; do timeout -k 10 60 scripts/expt/run scripts/expt/lib$v.so $v $nb >> gpurun_out/r3e2/expt.jsonl || exit 1; done; done
cat gpurun_out/r3e2/expt.jsonl
TAG=r3q2 PYTEST_K="multi_batch or wg_kernel or table_change or scenario" bash scripts/gpu_r3_quick.sh
