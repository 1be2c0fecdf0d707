#!/usr/bin/env python3
"""bench.py — pod-node evals/s and pods placed/s of the batched scheduling core on MI355X.

Metric (BASELINE.json): "pod-node evals/sec + pods placed/sec at 5k nodes, 1/2/4/8 MI355X".
A step = one pass of the hot path (filter -> prescore -> score -> select, i.e.
minisched/minisched.go:50-87 for every pod of a batch) over one batch of synthetic pods with
inputs already resident in HBM.

Modes
  batch       (default) BASELINE C3: 5,000 nodes x 100,000 pods per GPU. With N GPUs the pods
              are sharded (each rank its own 100k batch; no data-path collective) -> weak scaling.
  sequential  BASELINE C5: same sizes, one pod at a time with node-state commits.
  nodeshard   BASELINE C4 shape: the node table split over the ranks, per-shard best keys
              merged with an RCCL all-reduce(MAX), then decoded (--nodes 100000 --pods 1000000).

Launch: `python bench.py` (1 GPU) or
`python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N`.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "pod-node evals/sec + pods placed/sec at 5k nodes, 1/2/4/8 MI355X"
VALU_PEAK_LANE_OPS = 157.3e12 / 2  # MI355X_MICROARCH.md: FP32 vector peak 157.3 TFLOPS = 2 x lane-ops/s
HBM_PEAK = 8.0e12                  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# IDENT scan: per node word and pod pair one v_xor_b32 (all-VGPR form), and one
# v_pk_minimum3_f16 per two words -> 3 wave-instructions per 4 x 64 (pod, node) pairs
LANE_OPS_PER_EVAL = 0.75
# measured issue ceiling of exactly that instruction mix (2 x v_xor_b32 v,v + 1 v_pk_minimum3_f16,
# 8 waves per SIMD): scripts/ubench_valu3.hip -> profiles/r1_ubench_valu3.jsonl
UBENCH = ROOT / "profiles" / "r1_ubench_valu3.jsonl"
UBENCH_OP = "v_xor_b32 vv x2 + v_pk_minimum3_f16"
N_SIMD = 256 * 4


def batch_kernel_label(n_nodes, n_pods, shard, cus):
    """The kernel msh_kernels.hip launch_ident_dyn_t dispatches for this batch (default knobs):
    one pair range per wave (ident_wave_kernel, 256-thread workgroups; rounds of at most 8
    pairs) when the table is one 64,512-node compute tile and every wave of the chip gets at
    most 64 rounds; otherwise the work-queue kernel, in its MULTI form for tables of several
    tiles."""
    sh = str(shard).lower()
    pairs, full = (n_pods + 1) // 2, cus * 32
    wave_range = os.environ.get("MSH_WAVE_RANGE", "1").strip() not in ("0", "")
    if wave_range and n_nodes <= 64512 and 0 < pairs <= 8 * 64 * full:
        waves = min(full, -(-pairs // (4 if pairs < 4 * full else 7)))
        longest = -(-pairs // waves)
        rounds = -(-longest // 8)
        return f"ident_wave_kernel<8, {sh}, {-(-longest // rounds)}, 256>"
    return f"ident_dyn_kernel<8, {sh}, 1024, false, {str(n_nodes > 64512).lower()}>"


def measured_int_valu_ceiling() -> float | None:
    """Lane-ops/s of the scan's instruction mix at the best measured occupancy."""
    try:
        rows = [json.loads(l) for l in UBENCH.read_text().splitlines() if l.startswith("{")]
        ipc = max(r["wave_instr_per_simd_cycle@2.4GHz"] for r in rows if r.get("op") == UBENCH_OP)
        return ipc * 2.4e9 * N_SIMD * 64
    except Exception:
        return None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--mode", choices=["batch", "sequential", "nodeshard"], default="batch")
    ap.add_argument("--nodes", type=int, default=None)
    ap.add_argument("--pods", type=int, default=None, help="pods per GPU (batch/sequential) or total (nodeshard)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (0 = skip)")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--streams", type=int, default=2,
                    help="batch mode: independent batches pipelined over this many HIP streams")
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # the rank's device first, so the process group (RCCL) binds its communicator to it
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", init_method="env://")

    build = importlib.import_module("mini-kube-scheduler_amd.build")
    if not build.LIB.exists():
        build.build()
    msh = importlib.import_module("mini-kube-scheduler_amd")
    synth = importlib.import_module("mini-kube-scheduler_amd.synthetic")

    mode = args.mode
    if mode == "nodeshard":
        n_total = args.nodes or 100_000
        p_total = args.pods or 1_000_000
    else:
        n_total = args.nodes or 5_000
        p_total = args.pods or 100_000

    D = importlib.import_module("mini-kube-scheduler_amd.distributed")
    ctx = msh.DeviceContext(local)
    ctx.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER], [msh.ScorePluginConfig(msh.NODE_NUMBER, 1)])
    unsched, node_digit = synth.make_nodes(n_total)[1:]
    # Batch mode pipelines consecutive, independent batches over `nstreams` HIP streams (each with
    # its own pod batch and output buffers): a launch reaches the 8 XCDs up to ~4.5 us apart
    # (scripts/stamps_dyn.py), and on one stream every batch pays that skew plus the slowest XCD's
    # tail before the next may start. Sequential mode carries node state from batch to batch and
    # node-shard mode has a collective per step: both stay on one stream.
    nstreams = args.streams if mode == "batch" else 1
    sharded = None
    if mode == "nodeshard":
        sharded = D.NodeShardedScheduler(ctx, unsched, node_digit, world, rank)
        node_base = sharded.shard.lo
        pod_digit, pod_tol = synth._make_pods_fast(p_total, synth.SEED)[1:]
        batches = [(pod_digit, pod_tol)]
    else:
        ctx.upload_nodes(unsched, node_digit)
        node_base = 0
        # pod-sharded weak scaling: rank r owns pods [r*P*S, (r+1)*P*S) of one global stream,
        # split into S batches of P pods (one per stream)
        pd_all, pt_all = synth._make_pods_fast(p_total * world * nstreams, synth.SEED)[1:]
        batches = []
        for i in range(nstreams):
            lo = (rank * nstreams + i) * p_total
            batches.append((np.ascontiguousarray(pd_all[lo:lo + p_total]), np.ascontiguousarray(pt_all[lo:lo + p_total])))
    p = len(batches[0][0])
    bufs = []
    for pod_digit, pod_tol in batches:
        bufs.append({"pd": torch.from_numpy(pod_digit).to(dev), "pt": torch.from_numpy(pod_tol).to(dev),
                     "idx": torch.empty(p, dtype=torch.int32, device=dev),
                     "score": torch.empty(p, dtype=torch.int64, device=dev),
                     "status": torch.empty(p, dtype=torch.int32, device=dev),
                     "keys": torch.zeros(2 * p, dtype=torch.int32, device=dev)})
    klen = ctx.shard_keys_len(p) if mode == "nodeshard" else 0  # int32 keys one step all-reduces
    main_stream = torch.cuda.current_stream(dev)
    streams = [main_stream] + [torch.cuda.Stream(dev) for _ in range(nstreams - 1)]

    def step(k, ev0=None, ev1=None, single=False):
        b = bufs[0] if single else bufs[k % nstreams]
        st = main_stream if single else streams[k % nstreams]
        sh = st.cuda_stream
        if ev0 is not None:
            ev0.record(st)
        if mode == "batch":
            ctx.schedule_batch_device(p, b["pd"].data_ptr(), b["pt"].data_ptr(), b["idx"].data_ptr(),
                                      b["score"].data_ptr(), b["status"].data_ptr(), sh)
        elif mode == "sequential":
            ctx.schedule_sequential_device(p, b["pd"].data_ptr(), b["pt"].data_ptr(), 0, b["idx"].data_ptr(),
                                           b["score"].data_ptr(), b["status"].data_ptr(), sh)
        else:
            ctx.shard_keys_device(p, b["pd"].data_ptr(), b["pt"].data_ptr(), node_base, b["keys"].data_ptr(), sh)
        if ev1 is not None:
            ev1.record(st)
        if mode == "nodeshard":  # RCCL all-reduce(MAX) of the per-shard keys, then decode
            D.merge_shard_keys_(b["keys"][:klen])
            ctx.decode_keys_device(p, b["pd"].data_ptr(), b["pt"].data_ptr(), b["keys"].data_ptr(), b["idx"].data_ptr(),
                                   b["score"].data_ptr(), b["status"].data_ptr(), sh)

    def fork():  # the side streams start after everything already queued on the main stream
        ev = torch.cuda.Event()
        ev.record(main_stream)
        for st in streams[1:]:
            st.wait_event(ev)

    def join():
        for st in streams[1:]:
            ev = torch.cuda.Event()
            ev.record(st)
            main_stream.wait_event(ev)

    fork()
    for k in range(args.warmup):
        step(k)
    join()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()

    # Device time from HIP events on the main stream bracketing the whole timed region (side
    # streams fork from / join into it), divided by K: the interval at which batches complete.
    # No event between launches: an event record is itself a barrier + timestamp packet that
    # costs ~3.5 us of GPU time and breaks back-to-back dispatch (scripts/host_overhead.py).
    # Node-shard steps hold an RCCL all-reduce and a decode launch too, so there the shard kernel
    # is bracketed per step.
    per_step = mode == "nodeshard"
    evs = ([(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
           if per_step else [(None, None)] * args.steps)
    r0, r1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    r0.record(main_stream)
    fork()
    for k, (e0, e1) in enumerate(evs):
        step(k, e0, e1)
    join()
    r1.record(main_stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if per_step:
        kernel_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in evs]))
    else:
        kernel_ms = r0.elapsed_time(r1) / args.steps

    # Isolated launch time (outside the timed region): the same launches back to back on ONE
    # stream, which is what rocprofv3's per-kernel average measures.
    kernel_ms_isolated = kernel_ms
    if nstreams > 1:
        q0, q1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        q0.record(main_stream)
        for k in range(args.steps):
            step(k, single=True)
        q1.record(main_stream)
        torch.cuda.synchronize()
        kernel_ms_isolated = q0.elapsed_time(q1) / args.steps

    if world > 1:
        t = torch.tensor([elapsed, kernel_ms, kernel_ms_isolated], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms, kernel_ms_isolated = float(t[0]), float(t[1]), float(t[2])

    # ---- correctness spot-check of every buffer's last batch against the independent closed form ----
    check = "skipped"
    if rank == 0 and not args.no_check:
        sys.path.insert(0, str(ROOT / "tests"))
        from closed_form import closed_form  # independent checker, not the oracle
        ok = True
        for (pod_digit, pod_tol), b in zip(batches, bufs):
            ci, cs, cst = closed_form(unsched, node_digit, pod_digit, pod_tol)
            gi, gs, gst = b["idx"].cpu().numpy(), b["score"].cpu().numpy(), b["status"].cpu().numpy()
            ok = ok and (gi == ci).all() and (gs == cs).all() and (gst == cst).all()
        check = "bit-exact vs closed form" if ok else "MISMATCH"
    pod_digit, pod_tol = batches[0]

    n_local = ctx.n_nodes
    evals_total = float(n_total) * float(p if mode != "nodeshard" else p_total) * args.steps * (world if mode != "nodeshard" else 1)
    pods_total = float(p) * args.steps * (world if mode != "nodeshard" else 1)
    value = evals_total / elapsed
    ms_per_step = elapsed * 1e3 / args.steps

    # ---- roofline of the dominant kernel, per launch, from HIP events on the launch stream ----
    kern_s = kernel_ms * 1e-3
    evals_launch = float(n_local) * p
    lane_ops = LANE_OPS_PER_EVAL * evals_launch
    uniq_bytes = 2.0 * n_local + 18.0 * p           # node records + pod records + outputs, once
    survey_bytes = 2.0 * n_local * p + 18.0 * p      # SURVEY §8d accounting (counts L1/L2 re-reads)
    traffic = None
    pmc = ROOT / "profiles" / "pmc_latest.json"
    if pmc.exists():
        try:
            pj = json.loads(pmc.read_text())
            kj = pj.get("kernels", {}).get(mode, pj if pj.get("mode") == mode else {})
            if kj.get("nodes") == n_local and kj.get("pods") == p:
                traffic = kj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    ceiling = measured_int_valu_ceiling()
    if mode == "sequential":
        roofline = {
            "bound": "latency",
            "achieved": kernel_ms * 1e3 / p, "peak": None, "unit": "us/pod (serial)", "frac": None,
            "traffic": traffic, "kernel": "seq_kernel", "kernel_ms": kernel_ms,
            "note": "one pod at a time: scan + 2 wave reductions + 1 workgroup barrier per pod",
        }
    else:
        shard = mode == "nodeshard"
        kname = batch_kernel_label(n_local, p, shard, torch.cuda.get_device_properties(dev).multi_processor_count)
        iso_s = kernel_ms_isolated * 1e-3
        roofline = {
            "bound": "valu",
            "achieved": lane_ops / kern_s / 1e9,
            "peak": VALU_PEAK_LANE_OPS / 1e9,
            "unit": "Glane-op/s",
            "frac": lane_ops / kern_s / VALU_PEAK_LANE_OPS,
            "traffic": traffic,
            "kernel": kname,
            "kernel_ms": kernel_ms,
            "kernel_ms_note": (f"interval at which launches complete with {nstreams} streams in flight; "
                               "kernel_ms_isolated = the same launches back to back on one stream "
                               "(= rocprofv3's per-kernel average)") if nstreams > 1 else "one stream",
            "kernel_ms_isolated": kernel_ms_isolated,
            "frac_isolated": lane_ops / iso_s / VALU_PEAK_LANE_OPS,
            "lane_ops_per_eval": LANE_OPS_PER_EVAL,
            "measured_int_valu_ceiling": ceiling / 1e9 if ceiling else None,
            "frac_vs_measured_int_ceiling": (lane_ops / kern_s / ceiling) if ceiling else None,
            "hbm": {"bound": "hbm", "achieved": uniq_bytes / kern_s / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                    "frac": uniq_bytes / kern_s / HBM_PEAK, "bytes_per_launch": uniq_bytes,
                    "survey_8d_bytes_per_launch": survey_bytes,
                    "survey_8d_frac": survey_bytes / kern_s / HBM_PEAK},
        }

    cpu = cpu_omp = None
    if rank == 0 and args.cpu_seconds > 0:
        cpu = cpu_baseline(unsched, node_digit, pod_digit, pod_tol, args.cpu_seconds, mode)
        if mode != "sequential":
            cpu_omp = cpu_baseline(unsched, node_digit, pod_digit, pod_tol, args.cpu_seconds / 2, mode,
                                   threads=min(16, os.cpu_count() or 1))

    if rank == 0:
        if mode == "batch":
            wl = (f"C3 batched: {n_total} nodes x {p} pods per batch per GPU (pod-sharded over {world} GPU; "
                  f"{nstreams} independent batches in flight on {nstreams} HIP streams)")
        elif mode == "sequential":
            wl = f"C5 sequential-commit: {n_total} nodes x {p} pods per GPU, one pod at a time"
        else:
            wl = f"C4 node-sharded: {n_total} nodes over {world} GPU x {p_total} pods, RCCL allreduce(MAX) merge"
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "pod-node evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak" if mode != "nodeshard" else "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (splitmix64 seed 0x6d696e69: 10% unschedulable nodes, 1% non-digit pods, 5% tolerating)",
            "config": {"workload": wl, "nodes": n_total, "pods_per_step": int(p if mode != "nodeshard" else p_total),
                       "plugins": "filter=[NodeUnschedulable] prescore=[NodeNumber] score=[NodeNumber w=1]",
                       "parallelism": f"{'pod' if mode != 'nodeshard' else 'node'}-sharded x{world}",
                       "streams": nstreams},
            "pods_per_s": pods_total / elapsed,
            "check": check,
            "roofline": roofline,
            "cpu_baseline": cpu,
            "cpu_baseline_omp": cpu_omp,
        }
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(unsched, node_digit, pod_digit, pod_tol, budget_s: float, mode: str, threads: int = 1):
    """The C restatement (oracle/msh_oracle.c) on this host's cores, on a bounded sample of the
    same workload: pods in chunks against the full node table until the budget is spent."""
    O = importlib.import_module("oracle.oracle")
    build = importlib.import_module("mini-kube-scheduler_amd.build")
    build.build_oracle()
    n = len(unsched)
    p = len(pod_digit)
    chunk = min(2000 * threads, p)
    done, t, pos = 0, 0.0, 0
    # cycle over the batch (wrapping) until the budget is spent: a 10-30 s sample
    while t < budget_s and p > 0:
        sl = slice(pos, min(pos + chunk, p))
        t0 = time.perf_counter()
        if mode == "sequential":
            O.c_schedule_sequential(unsched, node_digit, pod_digit[sl], pod_tol[sl])
        else:
            O.c_schedule_batch(unsched, node_digit, pod_digit[sl], pod_tol[sl], threads=threads)
        t += time.perf_counter() - t0
        done += sl.stop - sl.start
        pos = 0 if sl.stop >= p else sl.stop
    evals = float(n) * done
    return {"value": evals / t, "unit": "pod-node evals/s", "cores": threads, "kind": "port",
            "sample": f"{done} pods (cycling over the {p}-pod batch) x {n} nodes, C restatement "
                      f"({'scalar' if threads == 1 else f'OpenMP {threads} threads'}), {t:.2f} s; "
                      f"{os.cpu_count()} host CPUs visible",
            "pods_per_s": done / t}


if __name__ == "__main__":
    main()
