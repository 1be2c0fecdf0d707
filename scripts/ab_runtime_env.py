"""A/B: submission strategies and HIP runtime settings that change the host cost of a launch or
of the final synchronize.

The headline was host-launch bound: each variant runs bench.py in a child process
(C3, no extras, no CPU baseline) at the driver's K = 20 / W = 5 and at K = 200, and prints one JSON
line per run with ms_per_step and the event-timed launch interval. Usage on the GPU box:
    python scripts/ab_runtime_env.py [variant ...] > gpurun_out/ab_env.jsonl
VARIANTS set runtime environment variables; SUBMIT variants pass bench.py flags ("base" = the default, mt3).
"""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
SUBMIT = {
    "submit:python2": ["--submit", "python", "--streams", "2"],
    "submit:mt2": ["--submit", "mt", "--streams", "2"],
    "submit:mt3": ["--submit", "mt", "--streams", "3"],
    "submit:mt4": ["--submit", "mt", "--streams", "4"],
    "submit:mt6": ["--submit", "mt", "--streams", "6"],
}
# hardware queues per process (HIP's default 4) x lanes: (env, bench.py flags)
for hq in (4, 8, 16):
    for ln in (3, 4, 6):
        SUBMIT[f"hwq{hq}:mt{ln}"] = ({"GPU_MAX_HW_QUEUES": str(hq)}, ["--submit", "mt", "--streams", str(ln)])
VARIANTS = {
    "base": {},
    "dev_kernarg_0": {"HIP_FORCE_DEV_KERNARG": "0"},
    "dev_kernarg_1": {"HIP_FORCE_DEV_KERNARG": "1"},
    "hdp_flush_wa_0": {"DEBUG_CLR_KERNARG_HDP_FLUSH_WA": "0"},
    "kernarg_copy_opt_0": {"DEBUG_HIP_KERNARG_COPY_OPT": "0"},
    "skip_kernarg_copy": {"ROC_SKIP_KERNEL_ARG_COPY": "1"},
    "active_wait_0": {"ROC_ACTIVE_WAIT_TIMEOUT": "0"},
    "active_wait_100": {"ROC_ACTIVE_WAIT_TIMEOUT": "100"},
    "direct_dispatch_0": {"AMD_DIRECT_DISPATCH": "0"},
}
REPS = int(os.environ.get("REPS", 3))
only = sys.argv[1:]
for name, env in list(VARIANTS.items()) + list(SUBMIT.items()):
    if only and name not in only:
        continue
    for k, reps in ((20, REPS), (200, 1)):
        for rep in range(reps):
            if isinstance(env, tuple):
                ev, extra = env
            else:
                ev, extra = (env, []) if isinstance(env, dict) else ({}, env)
            e = dict(os.environ, **ev)
            cmd = [sys.executable, str(ROOT / "bench.py"), "--steps", str(k), "--warmup", "5",
                   "--no-extras", "--cpu-seconds", "0", *extra]
            try:
                r = subprocess.run(cmd, env=e, capture_output=True, text=True, timeout=120)
            except subprocess.TimeoutExpired:
                print(json.dumps({"variant": name, "k": k, "error": "timeout"}), flush=True)
                sys.exit(1)
            if r.returncode:
                print(json.dumps({"variant": name, "k": k, "rc": r.returncode, "err": r.stderr[-400:]}), flush=True)
                sys.exit(1)
            line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
            print(json.dumps({"variant": name, "env": ev, "args": extra, "k": k, "rep": rep,
                              "ms_per_step": line["ms_per_step"], "value": line["value"],
                              "kernel_ms": line["roofline"]["kernel_ms"],
                              "kernel_ms_isolated": line["roofline"]["kernel_ms_isolated"],
                              "check": line["check"]}), flush=True)
