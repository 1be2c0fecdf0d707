#!/usr/bin/env python3
"""bench.py — pod-node evals/s and pods placed/s of the batched scheduling core on MI355X.

Metric (BASELINE.json): "pod-node evals/sec + pods placed/sec at 5k nodes, 1/2/4/8 MI355X".
A step = one pass of the hot path (filter -> prescore -> score -> select, i.e.
minisched/minisched.go:50-87 for every pod of a batch) over one batch of synthetic pods with
inputs already resident in HBM.

Plugins: BASELINE.json configs[2]'s "nodenumber prescore/score + weighted NormalizeScore":
filter=[NodeUnschedulable], prescore=[NodeNumber], score=[NodeNumber weight 3, DefaultNormalizeScore]
(HEADLINE_WEIGHT / HEADLINE_NORM). This departs from BASELINE.md's plugin table (weight 1, and its C3 row's
"weight 3 + identity normalize"): DefaultNormalizeScore maps 10 to 100, so it is not an identity. The
reference's own w = 1 list without a normalizer, BASELINE.md's definition and round 4's `value`, runs on the
same launches and is reported beside it (c3_plugin_variants.reference_weight1_none); the two time alike.

Modes (the headline line)
  batch       (default) BASELINE C3: 5,000 nodes x 100,000 pods per batch per GPU, on the per-pair kernel
              (every (pod, node) pair's filter and score evaluated from the node's and the pod's own bits,
              32 pairs per 32-bit lane-op). With N GPUs the pods are sharded (each rank its own 100k
              batches; no data-path collective) -> weak scaling. The K steps are K independent batches
              (32 distinct pod batches, each with its own outputs, used in turn) submitted from one host
              thread on one HIP stream through msh_schedule_batches_device, MSH_BATCHES_PER_LAUNCH (32)
              batches per kernel launch: the submission a caller with several drained batches ready makes.
  sequential  BASELINE C5: same sizes, one pod at a time with node-state commits.
  nodeshard   BASELINE C4 shape: the node table split over the ranks, per-pod first keys of every
              shard merged with an RCCL all-reduce(MAX), then decoded (--nodes 100000 --pods 1000000).

With one GPU, rank 0 also measures, after the timed region, and reports as extra keys of the same
line: the reference's w = 1 list and MIN-MAX / REVERSE at w = 3 on the same launches; generic_kernel
(the explicit int64 score per pair, north_star's five stages) on the reference plugin list and on
NodeNumber + a DEFAULT-normalized score column; the node-table maintenance (f2: msh_patch_nodes and
msh_upload_nodes); C5 sequential; C4 (100k nodes x 1M pods) on one GPU; C2; and the host-buffer path
(e2e: the C-ABI call a cgo caller makes, PCIe included). Each is checked bit-exact against an
independent checker (tests/closed_form.py; a sampled direct evaluation for the score-column list).

Launch: `python bench.py` (1 GPU) or
`python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N`.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import ctypes
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
CLOCK_HZ = 2.4e9                   # MI355X_MICROARCH.md: max clock
HBM_PEAK = 8.0e12                  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
LANES_PER_SIMD_CYCLE = 32          # MI355X_MICROARCH.md: SIMD-32, a wave64 VALU instruction over 2 cycles
# pair_kernel's scan (msh_pair.hip): per 32-node word and 64-pod wave, v_bitop3 (X & nT) + 4 v_bitop3
# (the code-bit mismatches ORed in: dm') and half a v_bitop3 AND3 (two words' dm' into the group's match
# flag): 5.5 VALU per 32 x 64 pairs in the identity-like modes (NONE, DEFAULT); REVERSE / MINMAX add one
# v_bitop3 OR-accumulate of the feasible non-matches: 6.5
PAIR_VALU_PER_WORD = 5.5
PAIR_VALU_PER_WORD_KX = 6.5
# the LDS-staged form (pair_lds_kernel) tracks its first feasible node per lane: one v_bitop3 per
# group and block (nT & the scalar AND of the group's X words), 5.5 + 1/8 per word in NONE
PAIR_VALU_PER_WORD_LDS = 5.625
# REVERSE / MINMAX in the LDS-staged form: group 0 scanned first settles the first feasible non-match for
# nearly every wave, so the other groups drop that reduction (5.5), and with the tolerates compaction 7
# of a workgroup's 8 pod blocks fold X & nT into the first code compare (4.625)
PAIR_VALU_PER_WORD_LDS_KX = 4.625
# generic_kernel's main loop on the reference list (NodeNumber only, 32-bit keys; the ISA of
# generic_kernel<0, 0, false, 0, false>): per 16 nodes and 2 pod blocks, 32 v_bfe_u32 (the pod's one-hot
# code bit at the node's digit), 32 v_mad_u32_u24 (the lane's weighted key), 32 v_bitop3_b32
# (NodeUnschedulable clears an infeasible key), 16 v_max3_u32 (the running maximum), 2 x (v_cmp_gt_u32 +
# v_cndmask_b32) for the chunk and a v_mov_b64: 117 VALU per 32 pairs
GEN_VALU_PER_PAIR_REF = 117 / 32
# seq_kernel's scan (msh_seq.hip), per 32-node word and pod: v_xor + 3 v_bitop3 (the code compare) + one
# v_bitop3 (NodeUnschedulable): 5 VALU per 32 pairs
SEQ_VALU_PER_WORD = 5
PAIR_LDS_MAX_GROUPS = 128          # msh_pair.hip: tables the LDS-staged pair kernel takes (4-wave workgroups)
PAIR_LDS_BIG_GROUPS = 416          # ... and with 16-wave workgroups
PAIR_SLICE_LDS_GROUPS = 128        # msh_pair.hip: tables whose planes the slice kernel (pair_kernel) stages in LDS
PMC_FILE = ROOT / "profiles" / "r6_pmc_c3.json"
# The headline plugin set (BASELINE C3: "nodenumber prescore/score + weighted NormalizeScore"): the
# reference's filter and prescore lists, NodeNumber scored at weight 3 with upstream's
# helper.DefaultNormalizeScore (MaxNodeScore 100) as its NormalizeScore. The reference itself has no
# weight (minisched.go:187 "TODO: plugin weight") and no ScoreExtensions (nodenumber.go:98-100): its
# w = 1 / no-normalizer list is timed beside it (extras "reference_weight1_none").
HEADLINE_WEIGHT = 3
HEADLINE_NORM = 1  # msh_normalize: MSH_NORMALIZE_DEFAULT
NORM_NAMES = {0: "none", 1: "DefaultNormalizeScore", 2: "DefaultNormalizeScore(reverse)", 3: "min-max"}
VALU_PEAK_FILE = ROOT / "profiles" / "r4_ubench_valu.json"


def batch_kernel_label(n_nodes: int, n_pods: int, cus: int, kx: bool = False, shard: bool = False,
                       multi: bool = False, nb: int = 1) -> str:
    """The kernel msh_capi.cpp dispatches for a launch of nb batches of n_pods (msh_pair.hip
    launch_pair_t): pair_lds_kernel<SHARD, KX, W> (planes staged in LDS, W waves per workgroup) when the
    launch fills the chip, else pair_kernel<S, SHARD, KX> (S slice waves per 64-pod block); KX for
    REVERSE / MINMAX."""
    b = lambda v: str(v).lower()
    groups = max(-(-n_nodes // 1024) * 1024, 1024) // 256
    waves = -(-n_pods // 64) * (nb if multi else 1)
    if groups <= PAIR_LDS_MAX_GROUPS and waves >= cus * 64:
        return f"void msh::pair_lds_kernel<{b(shard)}, {b(kx)}, 4>"
    if PAIR_LDS_MAX_GROUPS < groups <= PAIR_LDS_BIG_GROUPS and waves >= cus * 2 * 16:  # 16-wave workgroups
        return f"void msh::pair_lds_kernel<{b(shard)}, {b(kx)}, 16>"
    sl = 1
    while sl < 4 and waves * sl < cus * 16 and groups >= 4 * sl:
        sl *= 2
    # the last two parameters: the commit epilogue (sequential mode only) and the descriptor count of the
    # argument block (1 for a one-batch launch, 32 otherwise)
    # planes staged in LDS (the last parameter) for tables up to PAIR_SLICE_LDS_GROUPS groups
    return (f"void msh::pair_kernel<{sl}, {b(shard)}, {b(kx)}, false, {32 if multi and nb > 1 else 1}, "
            f"{b(groups <= PAIR_SLICE_LDS_GROUPS)}>")


def seq_shape(n_nodes: int, cap: bool = False):
    """seq_kernel's register layout for a table (launch_sequential): words per lane RS, scanning waves NW."""
    words = max(-(-n_nodes // 1024) * 1024, 1024) // 32
    rs = lambda nw: -(-words // (nw * 64))
    nw = 1 if rs(1) <= (16 if cap else 4) else 4 if rs(4) <= 4 else (16 if cap else 15)
    r = rs(nw)
    rsv = {1: [1, 2, 3, 4, 6, 8, 12, 16] if cap else [1, 2, 3, 4], 4: [2, 4]}.get(nw, [4, 8] if cap else [4, 8, 12])
    return next(v for v in rsv if r <= v), nw


def seq_kernel_label(n_nodes: int, cap: bool = False, kx: bool = False) -> str:
    r, nw = seq_shape(n_nodes, cap)
    if cap and nw == 1:  # msh_seq_cap.hip: one wave, 4 pods per step, counts in LDS, availability planes
        return f"void msh::seq_capu_kernel<{r}, {str(kx).lower()}, 4>"
    u = 1 if cap else 4  # SEQ_AHEAD: pods decided per step without a capacity
    # the last parameter: pod waves per pod-block workgroup (msh_internal.h SEQ_POD_WAVES, 1)
    return f"void msh::seq_kernel<{r}, {nw}, {str(kx).lower()}, {str(cap).lower()}, {u}, 1>"


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
    ap.add_argument("--no-extras", action="store_true", help="skip the secondary configs (one GPU only)")
    ap.add_argument("--submit", choices=["multi", "single"], default="multi",
                    help="batch mode: the K steps through msh_schedule_batches_device, 32 batches per launch "
                         "(default), or (A/B) one msh_schedule_batch_device launch per step; one host thread "
                         "and one HIP stream either way")
    return ap.parse_args()


def load_json(path: Path):
    try:
        return json.loads(path.read_text())
    except Exception:
        return None


class Streams:
    """Consecutive independent batches over `ns` HIP streams forked from / joined into the main one."""

    def __init__(self, torch, dev, ns):
        self.torch = torch
        self.main = torch.cuda.current_stream(dev)
        self.all = [self.main] + [torch.cuda.Stream(dev) for _ in range(ns - 1)]
        # fork / join events made once and reused: a torch Event creates its HIP event on its first
        # record, a few microseconds that would otherwise land inside every timed region
        self.fork_ev = torch.cuda.Event()
        self.join_evs = [torch.cuda.Event() for _ in self.all[1:]]
        self.fork()
        self.join()
        torch.cuda.synchronize()

    def fork(self):
        self.fork_ev.record(self.main)
        for st in self.all[1:]:
            st.wait_event(self.fork_ev)

    def join(self):
        for st, ev in zip(self.all[1:], self.join_evs):
            ev.record(st)
            self.main.wait_event(ev)

    def time(self, launch, k: int) -> float:
        """ms per launch over k launches, launch(i, stream) alternating the streams, HIP events
        on the main stream around the whole region."""
        e0, e1 = self.torch.cuda.Event(enable_timing=True), self.torch.cuda.Event(enable_timing=True)
        e0.record(self.main)
        self.fork()
        for i in range(k):
            launch(i, self.all[i % len(self.all)].cuda_stream)
        self.join()
        e1.record(self.main)
        self.torch.cuda.synchronize()
        return e0.elapsed_time(e1) / k


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # MSH_BENCH_REHEARSE=1 (one-GPU rehearsal of the N>1 path only): every rank on device 0 and the
    # process group on gloo, since RCCL refuses two ranks on one GPU. Never set for measurements.
    rehearse = os.environ.get("MSH_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    # the rank's device first, so the process group (RCCL) binds its communicator to it
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("gloo" if rehearse else "nccl", init_method="env://")

    build = importlib.import_module("mini-kube-scheduler_amd.build")
    if not build.LIB.exists():
        build.build()
    msh = importlib.import_module("mini-kube-scheduler_amd")
    synth = importlib.import_module("mini-kube-scheduler_amd.synthetic")
    D = importlib.import_module("mini-kube-scheduler_amd.distributed")
    sys.path.insert(0, str(ROOT / "tests"))
    from closed_form import closed_form_modes  # independent checker, not the oracle

    mode = args.mode
    n_total = args.nodes or (100_000 if mode == "nodeshard" else 5_000)
    p_total = args.pods or (1_000_000 if mode == "nodeshard" else 100_000)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count

    ctx = msh.DeviceContext(local)
    ctx.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER],
                    [msh.ScorePluginConfig(msh.NODE_NUMBER, HEADLINE_WEIGHT, msh.Normalize(HEADLINE_NORM))])
    unsched, node_digit = synth.make_nodes(n_total)[1:]
    G = msh._native.BATCHES_PER_LAUNCH  # batches per msh_schedule_batches_device launch
    multi = mode == "batch" and args.submit == "multi"
    if mode == "nodeshard":
        sharded = D.NodeShardedScheduler(ctx, unsched, node_digit, world, rank)
        node_base = sharded.shard.lo
        batches = [tuple(synth._make_pods_fast(p_total, synth.SEED)[1:])]
        if world > 1 and not rehearse:
            # the library's own RCCL communicator (msh_comm_*): rank 0 makes the id and the process group
            # only ships its 128 bytes (a Go scheduler would use its own channel); every step then merges
            # inside msh_schedule_nodeshard_device
            idt = torch.zeros(msh._native.COMM_ID_BYTES, dtype=torch.uint8, device=dev)
            if rank == 0:
                idt.copy_(torch.tensor(list(msh.DeviceContext.comm_unique_id()), dtype=torch.uint8))
            dist.broadcast(idt, 0)
            ctx.comm_init(bytes(idt.cpu().tolist()), world, rank)
    else:
        ctx.upload_nodes(unsched, node_digit)
        node_base = 0
        # pod-sharded weak scaling: rank r owns pods [r*P*B, (r+1)*P*B) of one global stream, split
        # into B distinct batches of P pods (batch mode: B = 32, step i schedules batch i mod 32)
        nb = G if mode == "batch" else 1
        pd_all, pt_all = synth._make_pods_fast(p_total * world * nb, synth.SEED)[1:]
        batches = []
        for i in range(nb):
            lo = (rank * nb + i) * p_total
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
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    # the msh_batch descriptors of the 32 batches, built once (host memory, read at each call)
    descs = ctx.batch_descs([(p, b["pd"].data_ptr(), b["pt"].data_ptr(), b["idx"].data_ptr(), b["score"].data_ptr(),
                              b["status"].data_ptr()) for b in bufs])
    fast, handle = ctx._fast, ctx._hv()
    batch_args = [(handle, p, b["pd"].data_ptr(), b["pt"].data_ptr(), b["idx"].data_ptr(), b["score"].data_ptr(),
                   b["status"].data_ptr(), sh or None) for b in bufs]
    descs_addr = __import__("ctypes").addressof(descs)

    def submit(k: int) -> None:
        """Steps 0..k-1 of the current mode, in order, on `stream` (one host thread)."""
        if mode == "batch" and multi:
            for i0 in range(0, k, G):  # batch i of a launch = buffer i (launches start at multiples of G)
                rc = fast.schedule_batches_device(handle, min(G, k - i0), descs_addr, sh or None)
                if rc:
                    ctx._check(rc)
            return
        for i in range(k):
            b = bufs[i % len(bufs)]
            if mode == "batch":
                rc = fast.schedule_batch_device(*batch_args[i % len(bufs)])
                if rc:
                    ctx._check(rc)
            elif mode == "sequential":
                ctx.schedule_sequential_device(p, b["pd"].data_ptr(), b["pt"].data_ptr(), 0, b["idx"].data_ptr(),
                                               b["score"].data_ptr(), b["status"].data_ptr(), sh)
            elif not rehearse:  # per-shard keys, RCCL all-reduce(MAX) and decode, all inside the library
                rc = fast.schedule_nodeshard_device(handle, p, b["pd"].data_ptr(), b["pt"].data_ptr(), node_base,
                                                    b["idx"].data_ptr(), b["score"].data_ptr(), b["status"].data_ptr(),
                                                    sh or None)
                if rc:
                    ctx._check(rc)
            else:  # rehearsal (every rank on one GPU: no RCCL communicator): the keys merged over gloo
                ctx.shard_keys_device(p, b["pd"].data_ptr(), b["pt"].data_ptr(), node_base, b["keys"].data_ptr(), sh)
                D.merge_shard_keys_(b["keys"][:klen], stream=stream)
                ctx.decode_keys_device(p, b["pd"].data_ptr(), b["pt"].data_ptr(), b["keys"].data_ptr(),
                                       b["idx"].data_ptr(), b["score"].data_ptr(), b["status"].data_ptr(), sh)

    submit(args.warmup)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # ---- the timed region: barrier (N > 1) + synchronize, K steps, synchronize (+ barrier). Nothing
    # but the K steps between the clocks: no events (two event records cost ~15 us of a 40 us K = 20
    # region, profiles/ab/r3_k20_probe.jsonl); the device span is taken from an untimed repeat below ----
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    submit(args.steps)
    torch.cuda.synchronize()
    if world > 1:  # the barrier and a second synchronize only where there is a barrier
        dist.barrier()
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0

    # the same K steps again, untimed by the clock, between two events on the launch stream: the
    # device span of a region (reported beside the wall-clock figure, never as `value`)
    r0, r1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for e in (r0, r1):  # create the HIP events first (a torch Event makes its HIP event on first record)
        e.record(stream)
    torch.cuda.synchronize()
    r0.record(stream)
    submit(args.steps)
    r1.record(stream)
    torch.cuda.synchronize()
    region_ms = r0.elapsed_time(r1)

    # ---- the dominant kernel's launch duration, for the roofline: R launches back to back on the
    # stream the kernels run on, each timed by its own start / stop events recorded at the kernel's
    # start and completion (msh_timing_begin: hipExtLaunchKernelGGL events, the interval rocprofv3's
    # kernel trace averages); in batch mode the full 32-batch launches of the default submission ----
    R = 50 if mode != "nodeshard" else min(args.steps, 20)
    ctx.timing_begin(R)
    for _ in range(R):
        if mode == "batch" and multi:
            rc = fast.schedule_batches_device(handle, G, descs_addr, sh or None)
            if rc:
                ctx._check(rc)
        elif mode == "batch":
            rc = fast.schedule_batch_device(*batch_args[0])
            if rc:
                ctx._check(rc)
        elif mode == "sequential":
            b = bufs[0]
            ctx.schedule_sequential_device(p, b["pd"].data_ptr(), b["pt"].data_ptr(), 0, b["idx"].data_ptr(),
                                           b["score"].data_ptr(), b["status"].data_ptr(), sh)
        else:
            b = bufs[0]
            ctx.shard_keys_device(p, b["pd"].data_ptr(), b["pt"].data_ptr(), node_base, b["keys"].data_ptr(), sh)
    n_timed, tot_ms, max_ms = ctx.timing_end()
    launch_ms = tot_ms / max(n_timed, 1)
    batches_per_launch = G if (mode == "batch" and multi) else 1
    if mode == "nodeshard":  # the timed steps hold the all-reduce and the decode too: redo them after
        submit(1)
        torch.cuda.synchronize()

    if world > 1:
        t = torch.tensor([elapsed, launch_ms, region_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, launch_ms, region_ms = float(t[0]), float(t[1]), float(t[2])

    # ---- correctness of every buffer's last batch against the independent closed form ----
    check = "skipped"
    if rank == 0 and not args.no_check:
        ok = True
        for (pod_digit, pod_tol), b in zip(batches, bufs):
            want = closed_form_modes(unsched, node_digit, pod_digit, pod_tol, HEADLINE_WEIGHT, HEADLINE_NORM)
            got = (b["idx"].cpu().numpy(), b["score"].cpu().numpy(), b["status"].cpu().numpy())
            ok = ok and all((g == w).all() for g, w in zip(got, want))
        check = "bit-exact vs closed form" if ok else "MISMATCH"

    n_local = ctx.n_nodes
    evals_total = float(n_total) * float(p if mode != "nodeshard" else p_total) * args.steps * (world if mode != "nodeshard" else 1)
    pods_total = float(p) * args.steps * (world if mode != "nodeshard" else 1)
    value = evals_total / elapsed
    ms_per_step = elapsed * 1e3 / args.steps

    roofline = make_roofline(mode, n_local, p, launch_ms, batches_per_launch, cus)
    roofline["region_device_ms_per_step"] = region_ms / args.steps

    extras = {}
    if rank == 0 and world == 1 and not args.no_extras:
        extras = measure_extras(torch, dev, msh, synth, D, closed_form_modes, cus)

    cpu = cpu_omp = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:  # the contract: rank 0 at N=1 only
        pod_digit, pod_tol = batches[0]
        cpu = cpu_baseline(unsched, node_digit, pod_digit, pod_tol, args.cpu_seconds, mode)
        if mode != "sequential":
            cpu_omp = cpu_baseline(unsched, node_digit, pod_digit, pod_tol, args.cpu_seconds / 2, mode,
                                   threads=host_cpu_share())

    if rank == 0:
        if mode == "batch":
            wl = (f"C3 batched: {n_total} nodes x {p} pods per batch per GPU (pod-sharded over {world} GPU); "
                  + (f"the K batches through msh_schedule_batches_device, {G} per launch, one stream"
                     if multi else "one msh_schedule_batch_device launch per batch, one stream"))
        elif mode == "sequential":
            wl = f"C5 sequential-commit: {n_total} nodes x {p} pods per GPU, one pod at a time"
        else:
            wl = (f"C4 node-sharded: {n_total} nodes over {world} GPU x {p_total} pods, msh_schedule_nodeshard_device "
                  "(shard keys, RCCL allreduce(MAX) on the library's communicator, decode)")
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
            "dtype": "u32 (bit-sliced: 32 pod-node pairs per lane-op)",
            "data": "synthetic (splitmix64 seed 0x6d696e69: 10% unschedulable nodes, 1% non-digit pods, 5% tolerating)",
            "config": {"workload": wl, "nodes": n_total, "pods_per_step": int(p if mode != "nodeshard" else p_total),
                       "plugins": (f"filter=[NodeUnschedulable] prescore=[NodeNumber] score=[NodeNumber "
                                   f"w={HEADLINE_WEIGHT} normalize={NORM_NAMES[HEADLINE_NORM]}]"),
                       "parallelism": f"{'pod' if mode != 'nodeshard' else 'node'}-sharded x{world}",
                       "streams": 1, "submit": (f"multi ({G} batches per launch)" if multi else "single") if mode == "batch"
                       else "per step",
                       **({"rehearsal": "all ranks on cuda:0, gloo (not a measurement)"} if rehearse else {})},
            "pods_per_s": pods_total / elapsed,
            "check": check,
            "roofline": roofline,
            "cpu_baseline": cpu,
            "cpu_baseline_omp": cpu_omp,
        }
        line.update(extras)
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


def load_valu_peak():
    """The integer VALU issue rates measured on MI355X (scripts/ubench_valu_r4.hip ->
    profiles/r4_ubench_valu.json), wave64 instructions per SIMD per cycle at 8 waves per SIMD: the best
    VGPR-only form (the issue peak) and the cap with one SGPR operand."""
    d = load_json(VALU_PEAK_FILE) or {}
    return d.get("vgpr_only_max"), d


def plugin_tag(weight: int, norm: int) -> str:
    """The NodeNumber score entry as profiles/r6_pmc_c3.json records it (scripts/run_batch.py)."""
    return f"NodeNumber w={weight} norm={norm}"


def pmc_entry(key: str, kname: str, n_local: int, p: int, nb: int, plugins: str | None = None):
    """The profiles/r6_pmc_c3.json entry for this kernel, size, batch count and plugin list (None if
    it does not match what this run timed)."""
    e = (load_json(PMC_FILE) or {}).get("kernels", {}).get(key, {})
    ok = (e.get("kernel") == kname and e.get("nodes") == n_local and e.get("pods") == p
          and e.get("batches_per_launch", 1) == nb and (plugins is None or e.get("plugins") == plugins))
    return e if ok else None


def valu_roofline(kname, launch_ms, evals, model_lane_ops_per_eval, cus, entry, model_note):
    """VALU roofline of an integer kernel: the modelled lane-ops per launch (the kernel's per-pair
    instruction count x the pairs it evaluates) / the launch's duration, against the MI355X VALU peak
    (CUs x 4 SIMD x 32 lanes per cycle x 2.4 GHz); the counter form uses rocprofv3 SQ_INSTS_VALU x 64
    of the same kernel, size and batch count (profiles/r4_pmc_c3.json)."""
    launch_s = launch_ms * 1e-3
    peak = cus * 4 * LANES_PER_SIMD_CYCLE * CLOCK_HZ  # lane-ops/s
    ipc, vd = load_valu_peak()
    peak_meas = ipc * 4 * 64 * cus * CLOCK_HZ if ipc else None
    sgpr_cap = vd.get("sgpr_operand_max")
    model = evals * model_lane_ops_per_eval
    instr = entry.get("SQ_INSTS_VALU") if entry else None
    cnt = instr * 64 if instr else None
    return {
        "bound": "valu",
        "achieved": model / launch_s / 1e9,
        "peak": peak / 1e9,
        "unit": "Glane-op/s",
        "frac": model / launch_s / peak,
        "traffic": entry.get("hbm_bytes_per_launch_fetch_x2") if entry else None,
        "traffic_note": ("rocprofv3 2 x FETCH_SIZE + WRITE_SIZE per launch (KiB x 1024; FETCH_SIZE doubled as "
                         "MI355X_MICROARCH.md's HBM section prescribes for gfx950), same kernel, size, batches "
                         "and plugin list, separate --pmc passes"),
        "kernel": kname,
        "kernel_ms": launch_ms,
        "kernel_ms_note": ("mean duration of R back-to-back launches, each timed from the kernel's own start "
                           "to its completion (msh_timing_begin / _end: hipExtLaunchKernelGGL events), the "
                           "interval rocprofv3's kernel trace averages"),
        "lane_ops_per_eval_model": model_lane_ops_per_eval,
        "model": model_note,
        "lane_ops_per_eval_counter": cnt / evals if cnt else None,
        "frac_counter": cnt / launch_s / peak if cnt else None,
        "counter_source": (f"rocprofv3 SQ_INSTS_VALU x 64 per launch ({PMC_FILE.name})" if cnt
                           else "no PMC entry for this kernel, size and batch count"),
        "peak_note": "MI355X_MICROARCH.md: SIMD-32 (a wave64 VALU instruction over 2 cycles), 4 SIMD per CU, 2.4 GHz",
        "peak_measured_issue": peak_meas / 1e9 if peak_meas else None,
        "frac_of_measured_issue": model / launch_s / peak_meas if peak_meas else None,
        "peak_measured_note": ("the best integer VALU issue rate measured with VGPR operands only (8 waves per "
                               f"SIMD, {VALU_PEAK_FILE.name}): {ipc:.3f} wave-instr per SIMD-cycle; with one SGPR "
                               f"operand the same forms cap at {sgpr_cap:.3f}" if ipc and sgpr_cap else None),
        "sgpr_operand_cap": sgpr_cap * 4 * 64 * cus * CLOCK_HZ / 1e9 if sgpr_cap else None,
    }


def seq_pair_label(n_nodes: int, n_pods: int, cus: int, kx: bool = False) -> str:
    """The kernel of a no-capacity sequential launch (msh_capi.cpp msh_schedule_sequential_device, auto):
    pair_kernel<S, false, KX, true>, the scalar-plane per-pair kernel with the commit epilogue."""
    groups = max(-(-n_nodes // 1024) * 1024, 1024) // 256
    waves = -(-n_pods // 64)
    sl = 1
    while sl < 4 and waves * sl < cus * 16 and groups >= 4 * sl:
        sl *= 2
    return f"void msh::pair_kernel<{sl}, false, {str(kx).lower()}, true, 1, {str(groups <= PAIR_SLICE_LDS_GROUPS).lower()}>"


def make_roofline(mode, n_local, p, launch_ms, batches_per_launch, cus, serial=False, cap=0, form="pair"):
    """Roofline of the dominant kernel, per launch: algorithmic work of one launch / the launch's
    average duration, measured with HIP events at the kernel's start and completion (bench.py main),
    the quantity rocprofv3's per-kernel average reports."""
    launch_s = launch_ms * 1e-3
    if mode == "sequential" and not serial and not cap and form == "pair":
        # Without a capacity (auto): the per-pair kernel over the whole batch with the commit epilogue (each
        # wave adds its placed pods to the node counts, one device atomic per distinct node)
        kname = seq_pair_label(n_local, p, cus)
        n_pad = max(-(-n_local // 1024) * 1024, 1024)
        model = PAIR_VALU_PER_WORD * (n_pad / 32) * (-(-p // 64) * 64) / (float(n_local) * p)
        entry = pmc_entry("sequential_pair", kname, n_local, p, 1, plugin_tag(HEADLINE_WEIGHT, HEADLINE_NORM))
        out = valu_roofline(kname, launch_ms, float(n_local) * p, model, cus, entry,
                            f"{PAIR_VALU_PER_WORD} VALU per 32-node word and 64-pod wave (pair_kernel's scan, "
                            "msh_pair.hip); the commit epilogue is in the counter form")
        if entry and "SQ_WAVE_CYCLES" in entry:
            out["wait_any_frac_of_wave_cycles"] = entry.get("sq_wait_any_frac_of_wave_cycles")
            out["wave_cycles_per_wave"] = 4 * entry["SQ_WAVE_CYCLES"] / entry["SQ_WAVES"]
        out["bound_note"] = ("one 100k-pod batch per launch is latency-bound, not issue-bound: each wave lives for "
                             "thousands of cycles around one memory round trip in and the stores out (DESIGN.md "
                             "§4.2 LDSP, §9); the VALU fraction is not the binding limit here")
        return out
    if mode == "sequential" and not serial:
        # Without a capacity the pods run in blocks of consecutive pods, one workgroup each (a wave per
        # block walks its pods in order, every pod against the whole register-resident table): VALU-bound
        # over the chip. Model: 5 VALU per 32-node word and pod (the pair evaluation; the first-hit
        # reduction and the per-pod decode are in the counter form).
        kname = seq_kernel_label(n_local)
        r, nw = seq_shape(n_local)
        model = SEQ_VALU_PER_WORD * nw * 64 * r / float(n_local)
        return valu_roofline(kname, launch_ms, float(n_local) * p, model, cus,
                             pmc_entry("sequential", kname, n_local, p, 1, plugin_tag(HEADLINE_WEIGHT, HEADLINE_NORM)),
                             f"{SEQ_VALU_PER_WORD} VALU per 32-node word and pod (seq_kernel's scan: v_xor and three "
                             "v_bitop3 for the code compare, one v_bitop3 for NodeUnschedulable), over the "
                             f"{nw} x 64 lanes x {r} words of the register-resident table")
    if mode == "sequential":
        # One wave decides the pods in order; alone on its SIMD it issues about one instruction per
        # 4 cycles of any kind (MI355X_MICROARCH.md, 'vector-instruction ISSUE cost'), so the floor
        # of the per-pod latency is its instruction count (VALU + SALU, counted by rocprofv3 for
        # this kernel at C5) x 4 cycles at 2.4 GHz. That is an issue floor of the code as written,
        # not a hardware roofline: reported as issue_floor_frac, not frac.
        kname = seq_kernel_label(n_local, cap=cap > 0)
        entry = pmc_entry("sequential_capacity" if cap else "sequential_serial", kname, n_local, p, 1)
        instr = (entry.get("SQ_INSTS_VALU", 0) + entry.get("SQ_INSTS_SALU", 0)) / p if entry else None
        floor_us = instr * 4 / 2.4e3 if instr else None
        achieved = launch_ms * 1e3 / p
        return {"bound": "issue latency (one wave, serial)", "achieved": achieved, "unit": "us/pod",
                "issue_floor_us_per_pod": floor_us,
                "issue_floor_frac": floor_us / achieved if floor_us else None,
                "kernel": kname, "kernel_ms": launch_ms,
                "traffic": entry.get("hbm_bytes_per_launch") if entry else None,
                "instructions_per_pod": instr,
                "note": "a serial mode: the floor is the kernel's own instruction count per pod (rocprofv3 "
                        "SQ_INSTS_VALU + SQ_INSTS_SALU / pods) x 4 cycles / 2.4 GHz, not a hardware roofline"}
    nb = batches_per_launch
    kname = batch_kernel_label(n_local, p, cus, shard=mode == "nodeshard", multi=nb > 1, nb=nb)
    evals = float(n_local) * p * nb
    n_pad = max(-(-n_local // 1024) * 1024, 1024)
    # every 64-pod wave meets every 32-node word of the padded table once
    lds = "pair_lds_kernel" in kname
    per_word = PAIR_VALU_PER_WORD_LDS if lds else PAIR_VALU_PER_WORD
    model_per_eval = per_word * (n_pad / 32) * (-(-p // 64) * 64) / (float(n_local) * p)
    entry = pmc_entry("pair_multi" if nb > 1 else "pair_single", kname, n_local, p, nb,
                      plugin_tag(HEADLINE_WEIGHT, HEADLINE_NORM))
    out = valu_roofline(kname, launch_ms, evals, model_per_eval, cus, entry,
                        f"{per_word} VALU per 32-node word and 64-pod wave ({kname.split('<')[0][10:]}'s scan, "
                        "msh_pair.hip, the identity-like normalize modes: NONE, DefaultNormalizeScore): per "
                        "lane-op 32 (pod, node) pairs get NodeUnschedulable's "
                        f"verdict and NodeNumber's digit compare; lane-ops per eval = {per_word} x padded words x "
                        "padded pods / (n x p)")
    out["batches_per_launch"] = nb
    out["ms_per_batch"] = launch_ms / nb
    # HBM: the bit planes once (0.75 B per node: 6 planes of 32 nodes per 4 B), 2 B in + 16 B out per pod
    uniq = 0.75 * n_pad + 18.0 * p * nb
    out["hbm"] = {"bound": "hbm", "achieved": uniq / launch_s / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                  "frac": uniq / launch_s / HBM_PEAK, "bytes_per_launch": uniq,
                  "note": "unique algorithmic bytes: the table is read by every wave through the scalar "
                          "cache / L2, never re-fetched from HBM (traffic, above, is the counter)"}
    return out


def multi_launch_ms(torch, ctx, descs, nb, R, stream):
    """Mean kernel duration of R launches of nb batches (msh_timing_begin / _end), after 3 untimed."""
    for _ in range(3):
        ctx.schedule_batches_device(descs, nb, stream)
    torch.cuda.synchronize()
    ctx.timing_begin(R)
    for _ in range(R):
        ctx.schedule_batches_device(descs, nb, stream)
    n_t, tot, _ = ctx.timing_end()
    torch.cuda.synchronize()
    return tot / max(n_t, 1)


def median_us(fn, k: int) -> float:
    """Median host wall time of k calls of fn (after one untimed call), in microseconds."""
    fn()
    ts = []
    for _ in range(k):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e6


def measure_extras(torch, dev, msh, synth, D, closed_form_modes, cus):
    """Secondary BASELINE configs, the other plugin lists, the generic kernel, the node-table maintenance
    and the host-buffer path, each timed and checked bit-exact."""
    from closed_form import direct_plugins
    out = {}
    G = msh._native.BATCHES_PER_LAUNCH

    def dbufs(pd, pt):
        p = len(pd)
        return [torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev), torch.empty(p, dtype=torch.int32, device=dev),
                torch.empty(p, dtype=torch.int64, device=dev), torch.empty(p, dtype=torch.int32, device=dev)]

    def got(b):
        return tuple(t.cpu().numpy() for t in b[2:])

    def same(a, b):
        return all((x == y).all() for x, y in zip(a, b))

    def new_ctx(options=None):
        c = msh.DeviceContext(dev.index or 0, options)  # msh_options overrides (msh_create_ex), A/B only
        c.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER],
                      [msh.ScorePluginConfig(msh.NODE_NUMBER, HEADLINE_WEIGHT, msh.Normalize(HEADLINE_NORM))])
        return c

    S2 = Streams(torch, dev, 2)
    sh = torch.cuda.current_stream(dev).cuda_stream

    # ---- C3 (5k x 100k): 32 batches per launch, on several kernels and plugin lists ----
    n, p = 5000, 100_000
    u, nd = synth.make_nodes(n)[1:]
    pd_all, pt_all = synth._make_pods_fast(G * p, synth.SEED + 1)[1:]
    pods = [(np.ascontiguousarray(pd_all[i * p:(i + 1) * p]), np.ascontiguousarray(pt_all[i * p:(i + 1) * p]))
            for i in range(G)]
    bufs = [dbufs(*pp) for pp in pods]
    descs = msh.DeviceContext.batch_descs([(p, *[t.data_ptr() for t in b]) for b in bufs])

    def run_multi(ctx, R=20):
        for b in bufs:
            b[2].fill_(-7)
        return multi_launch_ms(torch, ctx, descs, G, R, sh)

    def check_all(weight=1, norm=0):
        return all(same(got(b), closed_form_modes(u, nd, pp[0], pp[1], weight, norm)) for b, pp in zip(bufs, pods))

    ctx = new_ctx()
    ctx.upload_nodes(u, nd)
    # the other NormalizeScore modes and the reference's own list (w = 1, no normalizer) on the same
    # 32-batch launches as the headline, each with its VALU roofline (the counter form from its own
    # profiles/r6_pmc_c3.json entry)
    variants = {}
    for name, key, weight, norm in (("reference_weight1_none", "pair_multi_ref", 1, 0),
                                    ("minmax_weight3", "pair_minmax", 3, 3),
                                    ("reverse_weight3", "pair_reverse", 3, 2)):
        ctx.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER],
                        [msh.ScorePluginConfig(msh.NODE_NUMBER, weight, msh.Normalize(norm))])
        ms = run_multi(ctx)
        kx = norm in (2, 3)
        kname = batch_kernel_label(n, p, cus, kx=kx, multi=True, nb=G)
        per_word = PAIR_VALU_PER_WORD_LDS_KX if kx else PAIR_VALU_PER_WORD_LDS
        model = per_word * (-(-n // 1024) * 1024 / 32) * (-(-p // 64) * 64) / (float(n) * p)
        rl = valu_roofline(kname, ms, float(n) * p * G, model, cus, pmc_entry(key, kname, n, p, G, plugin_tag(weight, norm)),
                           f"{per_word} VALU per 32-node word and 64-pod wave (pair_lds_kernel's scan in this mode)")
        variants[name] = {"plugins": f"score=[NodeNumber w={weight} normalize={NORM_NAMES[norm]}]",
                          "kernel": kname, "kernel_ms": ms,
                          "batches_per_launch": G, "ms_per_batch": ms / G, "evals_per_s": n * p * G / (ms * 1e-3),
                          "check": "bit-exact vs closed form" if check_all(weight, norm) else "MISMATCH",
                          "roofline": rl}
    out["c3_plugin_variants"] = variants
    ctx.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER],
                    [msh.ScorePluginConfig(msh.NODE_NUMBER, HEADLINE_WEIGHT, msh.Normalize(HEADLINE_NORM))])

    # ---- generic_kernel: an explicit int64 score per (pod, node) pair (north_star's five stages) ----
    gen = {}
    gctx = new_ctx({"batch_kernel": "generic"})  # every plugin list on generic_kernel (the reference list included)
    gctx.upload_nodes(u, nd)
    gctx.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER], [msh.ScorePluginConfig(msh.NODE_NUMBER, 1)])
    ms = run_multi(gctx, R=5)
    kname = "void msh::generic_kernel<0, 0, false, 0, false>"
    rl = valu_roofline(kname, ms, float(n) * p * G, GEN_VALU_PER_PAIR_REF, cus,
                       pmc_entry("generic_ref", kname, n, p, G),
                       "3.66 VALU per pair (generic_kernel's main loop, NodeNumber only, 32-bit keys: v_bfe_u32 and "
                       "v_mad_u32_u24 for the weighted key, v_bitop3 for NodeUnschedulable, half a v_max3 for the "
                       "running maximum, 3 VALU per 16-node chunk and block)")
    gen["reference_list"] = {"kernel": kname, "kernel_ms": ms, "batches_per_launch": G, "ms_per_batch": ms / G,
                             "evals_per_s": n * p * G / (ms * 1e-3), "pods_per_s": p * G / (ms * 1e-3),
                             "check": "bit-exact vs closed form" if check_all() else "MISMATCH", "roofline": rl}
    # the headline list on generic_kernel: the extents pass (NodeNumber's pair flags: v_alignbit + v_or per
    # pair, one v_bitop3 per node and wave) before the main pass
    gctx.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER],
                     [msh.ScorePluginConfig(msh.NODE_NUMBER, HEADLINE_WEIGHT, msh.Normalize(HEADLINE_NORM))])
    ms = run_multi(gctx, R=5)
    entry = pmc_entry("generic_hl", kname, n, p, G, plugin_tag(HEADLINE_WEIGHT, HEADLINE_NORM))
    gen["headline_list"] = {
        "kernel": kname, "plugins": f"score=[NodeNumber w={HEADLINE_WEIGHT} normalize={NORM_NAMES[HEADLINE_NORM]}]",
        "kernel_ms": ms, "batches_per_launch": G, "ms_per_batch": ms / G, "evals_per_s": n * p * G / (ms * 1e-3),
        "lane_ops_per_eval_counter": entry["SQ_INSTS_VALU"] * 64 / (float(n) * p * G) if entry else None,
        "check": "bit-exact vs closed form" if check_all(HEADLINE_WEIGHT, HEADLINE_NORM) else "MISMATCH"}
    col = (np.arange(n, dtype=np.int64) * 7919) % 1000 - 300
    plugins = [("NodeNumber", 1, 0), ("ScoreColumn0", 2, 1)]
    gctx.upload_score_column("ScoreColumn0", col)
    gctx.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER],
                     [msh.ScorePluginConfig(nm, w, msh.Normalize(m)) for nm, w, m in plugins])
    ms = run_multi(gctx, R=5)
    sample = slice(0, 1500)
    ok = all(same(tuple(x[sample] for x in got(b)),
                  direct_plugins(u, nd, pp[0][sample], pp[1][sample], plugins, {0: col}))
             for b, pp in list(zip(bufs, pods))[:2])
    kname = "void msh::generic_kernel<0, 0, false, 1, false>"
    entry = pmc_entry("generic_col", kname, n, p, G)
    gen["nodenumber_plus_default_column"] = {
        "kernel": kname, "plugins": "score=[NodeNumber w=1, ScoreColumn0 w=2 DefaultNormalizeScore]",
        "kernel_ms": ms, "batches_per_launch": G, "ms_per_batch": ms / G, "evals_per_s": n * p * G / (ms * 1e-3),
        "lane_ops_per_eval_counter": entry["SQ_INSTS_VALU"] * 64 / (float(n) * p * G) if entry else None,
        "check": "sampled (1,500 pods of 2 batches) bit-exact vs a direct evaluation" if ok else "MISMATCH"}
    # two normalizing columns: generic_kernel's general form (a runtime column count, double keys)
    col1 = (np.arange(n, dtype=np.int64) * 104729) % 101
    gctx.upload_score_column("ScoreColumn1", col1)
    plugins = [("NodeNumber", 1, 0), ("ScoreColumn0", 2, 1), ("ScoreColumn1", 1, 3)]
    gctx.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER],
                     [msh.ScorePluginConfig(nm, w, msh.Normalize(m)) for nm, w, m in plugins])
    ms = run_multi(gctx, R=3)
    ok = all(same(tuple(x[sample] for x in got(b)),
                  direct_plugins(u, nd, pp[0][sample], pp[1][sample], plugins, {0: col, 1: col1}))
             for b, pp in list(zip(bufs, pods))[:2])
    gen["two_normalizing_columns"] = {
        "kernel": "void msh::generic_kernel<0, 0, true, 2, true>",
        "plugins": "score=[NodeNumber w=1, ScoreColumn0 w=2 DefaultNormalizeScore, ScoreColumn1 w=1 min-max]",
        "kernel_ms": ms, "batches_per_launch": G, "ms_per_batch": ms / G, "evals_per_s": n * p * G / (ms * 1e-3),
        "check": "sampled (1,500 pods of 2 batches) bit-exact vs a direct evaluation" if ok else "MISMATCH"}
    # a column over the whole int32 range: no 32-bit bound on the totals, generic_kernel's 64-bit form
    wide = ((np.arange(n, dtype=np.int64) * 2654435761) % (1 << 32)) - (1 << 31)
    gctx.upload_score_column("ScoreColumn0", wide)
    for key, cn in (("wide_column_none", 0), ("wide_column_default", 1)):
        plugins = [("NodeNumber", 1, 0), ("ScoreColumn0", 1, cn)]
        gctx.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER],
                         [msh.ScorePluginConfig(nm, w, msh.Normalize(m)) for nm, w, m in plugins])
        ms = run_multi(gctx, R=5)
        ok = all(same(tuple(x[sample] for x in got(b)),
                      direct_plugins(u, nd, pp[0][sample], pp[1][sample], plugins, {0: wide}))
                 for b, pp in list(zip(bufs, pods))[:2])
        gen[key] = {"kernel": f"void msh::generic_kernel<0, 2, {'true' if cn == 0 else 'false'}, {0 if cn == 0 else 1}, false>",
                    "plugins": f"score=[NodeNumber w=1, ScoreColumn0 w=1 {NORM_NAMES[cn]}] (column over the whole int32 range)",
                    "kernel_ms": ms, "batches_per_launch": G, "ms_per_batch": ms / G,
                    "evals_per_s": n * p * G / (ms * 1e-3),
                    "check": "sampled (1,500 pods of 2 batches) bit-exact vs a direct evaluation" if ok else "MISMATCH"}
    out["generic"] = gen
    gctx.close()

    # ---- e2e: the host-buffer C-ABI call (msh_schedule_batch), PCIe in and out ----
    pd, pt = pods[0]
    want = closed_form_modes(u, nd, pd, pt, HEADLINE_WEIGHT, HEADLINE_NORM)
    hpd, hpt = msh.pinned_empty(p, np.int8), msh.pinned_empty(p, np.uint8)
    hpd[:], hpt[:] = pd, pt
    e2e = {}
    for name, args, outs in (("pinned", (hpd, hpt), (msh.pinned_empty(p, np.int32), msh.pinned_empty(p, np.int64),
                                                       msh.pinned_empty(p, np.int32))),
                             ("pageable", (pd, pt), (np.empty(p, np.int32), np.empty(p, np.int64), np.empty(p, np.int32))),
                             ("pinned_no_scores", (hpd, hpt), (msh.pinned_empty(p, np.int32), None,
                                                                msh.pinned_empty(p, np.int32)))):
        scores = outs[1] is not None  # ABI v4: out_score = NULL, scores not written (8 of 16 B per pod)
        for _ in range(5):
            ctx.schedule_batch(*args, out=outs, scores=scores)
        ts = []
        for _ in range(50):
            t0 = time.perf_counter()
            ctx.schedule_batch(*args, out=outs, scores=scores)
            ts.append(time.perf_counter() - t0)
        us = float(np.median(ts)) * 1e6
        ok = same(outs, want) if scores else ((outs[0] == want[0]).all() and (outs[2] == want[2]).all())
        e2e[name] = {"us_per_batch": us, "pods_per_s": p / (us * 1e-6), "evals_per_s": n * p / (us * 1e-6),
                     "check": "bit-exact vs closed form" if ok else "MISMATCH"}
    # t_e2e with the SoA pack: msh_pack_pods turns the pods' names and
    # tolerations (a names blob and toleration records, built once, untimed) into the page-locked
    # digit / tolerates columns, then the pinned call; the packed columns are checked too
    names, pdn, ptn = synth.make_pods(p)
    snap = importlib.import_module("mini-kube-scheduler_amd.snapshot")
    blob, off = snap._blob(names)
    N = msh._native
    keep = [b"node.kubernetes.io/unschedulable", b"Exists", b"", b"NoSchedule"]
    tol_idx = np.flatnonzero(ptn)
    tols = (N.Toleration * max(len(tol_idx), 1))(*[N.Toleration(*keep) for _ in tol_idx])
    tol_off = np.zeros(p + 1, np.int64)
    tol_off[1:] = np.cumsum(ptn.astype(np.int64))
    lib = N.lib()
    pack_args = (p, blob, N.ptr(off), ctypes.cast(tols, ctypes.POINTER(N.Toleration)), N.ptr(tol_off),
                 N.ptr(hpd), N.ptr(hpt))
    outs = (msh.pinned_empty(p, np.int32), msh.pinned_empty(p, np.int64), msh.pinned_empty(p, np.int32))
    ts_pack, ts_all = [], []
    for i in range(55):
        t0 = time.perf_counter()
        rc = lib.msh_pack_pods(*pack_args)
        t1 = time.perf_counter()
        ctx.schedule_batch(hpd, hpt, out=outs)
        t2 = time.perf_counter()
        if rc != 0:
            raise RuntimeError(f"msh_pack_pods: {rc}")
        if i >= 5:
            ts_pack.append(t1 - t0)
            ts_all.append(t2 - t0)
    ok = (hpd == pdn).all() and (hpt == ptn).all() and same(outs, closed_form_modes(u, nd, pdn, ptn, HEADLINE_WEIGHT, HEADLINE_NORM))
    e2e["pinned_with_pack"] = {"us_per_batch": float(np.median(ts_all)) * 1e6,
                               "pack_us": float(np.median(ts_pack)) * 1e6,
                               "check": "packed columns == generator, outputs bit-exact vs closed form" if ok
                               else "MISMATCH"}
    # the same, pipelined (msh_schedule_batch_async + msh_wait): batch i + 1 is packed into the second
    # set of page-locked buffers while batch i runs, the loop a cgo caller draining activeQ runs
    sets = [(msh.pinned_empty(p, np.int8), msh.pinned_empty(p, np.uint8),
             (msh.pinned_empty(p, np.int32), msh.pinned_empty(p, np.int64), msh.pinned_empty(p, np.int32)))
            for _ in range(2)]
    set_args = [(p, blob, N.ptr(off), ctypes.cast(tols, ctypes.POINTER(N.Toleration)), N.ptr(tol_off),
                 N.ptr(spd), N.ptr(spt)) for spd, spt, _ in sets]

    def pipelined(nb):
        rc = lib.msh_pack_pods(*set_args[0])
        prev = ctx.schedule_batch_async(sets[0][0], sets[0][1], sets[0][2])
        for i in range(1, nb):
            k = i % 2  # last used by batch i - 2, waited for in iteration i - 1
            rc |= lib.msh_pack_pods(*set_args[k])
            t = ctx.schedule_batch_async(sets[k][0], sets[k][1], sets[k][2])
            ctx.wait(prev)
            prev = t
        ctx.wait(prev)
        if rc:
            raise RuntimeError("msh_pack_pods failed")

    pipelined(10)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        pipelined(40)
        ts.append((time.perf_counter() - t0) / 40)
    want_n = closed_form_modes(u, nd, pdn, ptn, HEADLINE_WEIGHT, HEADLINE_NORM)
    ok = all((spd == pdn).all() and (spt == ptn).all() and same(o, want_n) for spd, spt, o in sets)
    e2e["pinned_with_pack_pipelined"] = {
        "us_per_batch": float(np.median(ts)) * 1e6, "pods_per_s": p / float(np.median(ts)),
        "evals_per_s": n * p / float(np.median(ts)), "batches_per_run": 40,
        "check": "packed columns == generator, outputs bit-exact vs closed form" if ok else "MISMATCH",
        "note": "msh_pack_pods of batch i + 1 overlaps batch i on the device (msh_schedule_batch_async / "
                "msh_wait, two sets of page-locked buffers); median of 5 runs of 40 batches"}
    e2e["note"] = ("msh_schedule_batch from host buffers, synchronous, median of 50 calls (C3): the kernel "
                   "reads the pod columns from and writes the outputs into page-locked host memory over PCIe; "
                   "'pinned' = buffers from msh_host_alloc (no host copy), 'pageable' = numpy arrays (staged "
                   "through the ctx's page-locked buffer, copies split over host threads); 'pinned_with_pack' "
                   "adds msh_pack_pods (names + tolerations -> the digit / tolerates columns, one host "
                   "thread) in front of the pinned call; 'pinned_no_scores' passes out_score = NULL")
    out["e2e"] = e2e

    # ---- C5: 5k x 100k sequential commit (one launch = the whole 100k-pod batch), as the product runs
    # it (no capacity: blocks of consecutive pods, one workgroup each, every block in order) and with
    # the whole batch in one workgroup (MSH_SEQ_SPLIT=serial: the literal serial order, latency-bound);
    # each launch timed by its own kernel events ----
    b = dbufs(pd, pt)

    def c5(c, R):
        """Mean kernel duration of R launches (their own events), then the wall clock of R more back to back
        between two synchronizes (per launch: launch gaps and host submission included); the counts of
        all 2R launches checked."""
        seq = lambda: c.schedule_sequential_device(p, b[0].data_ptr(), b[1].data_ptr(), 0,
                                                   *[t.data_ptr() for t in b[2:]], sh)
        for _ in range(1 if R < 10 else 5):
            seq()
        torch.cuda.synchronize()
        c.reset_node_pod_counts()
        c.timing_begin(R)
        for _ in range(R):
            seq()
        n_t, tot, _ = c.timing_end()
        torch.cuda.synchronize()
        ms = tot / max(n_t, 1)
        t0 = time.perf_counter()
        for _ in range(R):
            seq()
        torch.cuda.synchronize()
        wall_ms = (time.perf_counter() - t0) * 1e3 / R
        counts = c.node_pod_counts()
        g = got(b)
        placed = g[2] == 0
        ok = same(g, want) and (counts == 2 * R * np.bincount(g[0][placed], minlength=n)).all()
        return ms, wall_ms, ok

    forms = {"pair": "no capacity (auto): the per-pair batch kernel over the whole batch with the commit epilogue "
                     "(each wave adds its placed pods to the node counts, one device atomic per distinct node); "
                     "no commit feeds a later decision, so the placements are the batch's",
             "blocks": "no capacity (msh_options.seq_split blocks): blocks of 64 consecutive pods, one workgroup "
                       "each, the pods within a block in order; node counts added by device atomics",
             "serial": "one workgroup walks all 100,000 pods in order"}
    for key, form, R in (("c5_sequential", "pair", 100), ("c5_sequential_blocks", "blocks", 100),
                         ("c5_sequential_serial", "serial", 3)):
        c = ctx if form == "pair" else new_ctx({"seq_split": form})
        if form != "pair":
            c.upload_nodes(u, nd)
        ms, wall_ms, ok = c5(c, R)
        kname = seq_pair_label(n, p, cus) if form == "pair" else seq_kernel_label(n)
        out[key] = {"kernel": kname, "ms_per_step": ms, "us_per_pod": ms * 1e3 / p,
                    "wall_ms_per_launch_back_to_back": wall_ms,
                    "pods_per_s": p / (ms * 1e-3), "evals_per_s": n * p / (ms * 1e-3), "form": forms[form],
                    "check": (f"seq == batch (closed form), node counts == {2 * R} x placements" if ok else "MISMATCH"),
                    "roofline": make_roofline("sequential", n, p, ms, 1, cus, serial=form == "serial", form=form)}
        c.close()

    # ---- C5 with a capacity (15 pods per node, the reference list): the one sequential form in which a
    # commit changes a later decision (a node that fills becomes infeasible), so one workgroup walks all
    # 100,000 pods in order; the counts are reset before each launch (each sees the same empty cluster) ----
    from closed_form import closed_form_capacity
    CAP = 15
    cc = new_ctx()
    cc.set_plugins([msh.NODE_UNSCHEDULABLE], [msh.NODE_NUMBER], [msh.ScorePluginConfig(msh.NODE_NUMBER, 1)])
    cc.upload_nodes(u, nd)
    seqc = lambda: cc.schedule_sequential_device(p, b[0].data_ptr(), b[1].data_ptr(), CAP,
                                                 *[t.data_ptr() for t in b[2:]], sh)
    cc.reset_node_pod_counts()
    seqc()
    torch.cuda.synchronize()
    R, tot = 3, 0.0
    for _ in range(R):
        cc.reset_node_pod_counts()
        cc.timing_begin(1)
        seqc()
        n_t, t_ms, _ = cc.timing_end()
        tot += t_ms / max(n_t, 1)
    ms = tot / R
    wi, ws, wst, wcounts = closed_form_capacity(u, nd, pd, pt, 1, CAP)
    ok = same(got(b), (wi, ws, wst)) and (cc.node_pod_counts() == wcounts).all() and wcounts.max() == CAP
    rl = make_roofline("sequential", n, p, ms, 1, cus, serial=True, cap=CAP)
    out["c5_sequential_capacity"] = {
        "kernel": seq_kernel_label(n, cap=True), "plugins": "score=[NodeNumber w=1] (the reference list)",
        "max_pods_per_node": CAP, "ms_per_step": ms, "us_per_pod": ms * 1e3 / p, "pods_per_s": p / (ms * 1e-3),
        "evals_per_s": n * p / (ms * 1e-3),
        "form": "one workgroup walks all 100,000 pods in order; a commit that fills a node makes it infeasible "
                "for the next pod",
        "check": (f"bit-exact vs an independent serial capacity simulation (tests/closed_form.py), node counts "
                  f"equal, fullest node = {CAP}" if ok else "MISMATCH"),
        "roofline": rl}
    cc.close()

    # ---- f2: node-table maintenance (an informer Update / Add, eventhandler.go:37-57, replacing the
    # per-cycle LIST of minisched.go:40), host wall time of the synchronous call, median of 50 ----
    tm = {}
    for n_t in (5000, 100_000):
        u_t, nd_t = synth.make_nodes(n_t)[1:]
        ctx = new_ctx()
        ctx.upload_nodes(u_t, nd_t)
        row = {"full_upload_us": median_us(lambda: ctx.upload_nodes(u_t, nd_t), 50)}
        rng = np.random.default_rng(n_t)
        for k in (1, 64, 1024):
            idx = rng.choice(n_t, k, replace=False).astype(np.int32)
            flip = [(1 - u_t[idx]).astype(np.uint8), u_t[idx].astype(np.uint8)]
            state = [0]

            def patch():
                ctx.patch_nodes(idx, flip[state[0]], nd_t[idx])
                state[0] ^= 1

            row[f"patch_{k}_nodes_us"] = median_us(patch, 50)
            if state[0]:  # an odd number of flips: flip back to the uploaded table
                patch()
        # the table after an even number of flips is the uploaded one: check a batch against it
        pd_t, pt_t = synth._make_pods_fast(4096, synth.SEED)[1:]
        ok = same(ctx.schedule_batch(pd_t, pt_t), closed_form_modes(u_t, nd_t, pd_t, pt_t, HEADLINE_WEIGHT, HEADLINE_NORM))
        row["check"] = "bit-exact vs closed form after the flips" if ok else "MISMATCH"
        tm[f"{n_t}_nodes"] = row
        ctx.close()
    tm["note"] = ("msh_patch_nodes of up to 64 nodes: one launch that copies the published table version and "
                  "rebuilds only the patched 32-node words' planes; more nodes: copy + scatter + the O(N) prep; "
                  "msh_upload_nodes: the H2D copy of 2 B/node + the prep")
    out["table_maintenance"] = tm

    # ---- C2: 1k x 10k, one launch per batch over two streams ----
    n2, p2 = 1000, 10_000
    u2, nd2 = synth.make_nodes(n2)[1:]
    pd2, pt2 = synth._make_pods_fast(2 * p2, synth.SEED)[1:]
    ctx = new_ctx()
    ctx.upload_nodes(u2, nd2)
    pairs2 = [(np.ascontiguousarray(pd2[:p2]), np.ascontiguousarray(pt2[:p2])),
              (np.ascontiguousarray(pd2[p2:]), np.ascontiguousarray(pt2[p2:]))]
    bs = [dbufs(*pp) for pp in pairs2]
    launch = lambda i, sh: ctx.schedule_batch_device(p2, *[t.data_ptr() for t in bs[i % 2]], sh)
    S2.time(launch, 4)
    ms = S2.time(launch, 100)
    ok = all(same(got(b2), closed_form_modes(u2, nd2, pp[0], pp[1], HEADLINE_WEIGHT, HEADLINE_NORM)) for b2, pp in zip(bs, pairs2))
    out["c2"] = {"kernel": batch_kernel_label(n2, p2, cus), "ms_per_step": ms, "evals_per_s": n2 * p2 / (ms * 1e-3),
                 "streams": 2, "check": "bit-exact vs closed form" if ok else "MISMATCH"}
    ctx.close()

    # ---- C4 on one GPU: 100k nodes x 1M pods, whole table, and one-rank node-shard keys + decode ----
    n4, p4 = 100_000, 1_000_000
    u4, nd4 = synth.make_nodes(n4)[1:]
    pd4, pt4 = synth._make_pods_fast(p4, synth.SEED)[1:]
    want4 = closed_form_modes(u4, nd4, pd4, pt4, HEADLINE_WEIGHT, HEADLINE_NORM)
    ctx = new_ctx()
    ctx.upload_nodes(u4, nd4)
    b4 = dbufs(pd4, pt4)
    s1 = Streams(torch, dev, 1)
    launch = lambda i, sh: ctx.schedule_batch_device(p4, *[t.data_ptr() for t in b4], sh)
    s1.time(launch, 1)
    ms_b = s1.time(launch, 5)
    ok_b = same(got(b4), want4)
    keys = torch.empty(ctx.shard_keys_len(p4), dtype=torch.int32, device=dev)

    def shard_step(i, sh):
        ctx.shard_keys_device(p4, b4[0].data_ptr(), b4[1].data_ptr(), 0, keys.data_ptr(), sh)
        D.merge_shard_keys_(keys)  # world 1: no collective
        ctx.decode_keys_device(p4, b4[0].data_ptr(), b4[1].data_ptr(), keys.data_ptr(), *[t.data_ptr() for t in b4[2:]], sh)

    for t in b4[2:]:
        t.fill_(-7)
    s1.time(shard_step, 1)
    ms_s = s1.time(shard_step, 5)
    ok_s = same(got(b4), want4)
    out["c4_one_gpu"] = {
        "batch": {"kernel": batch_kernel_label(n4, p4, cus), "ms_per_step": ms_b, "evals_per_s": n4 * p4 / (ms_b * 1e-3),
                  "check": "bit-exact vs closed form" if ok_b else "MISMATCH"},
        "node_shard_keys_plus_decode": {"kernel": batch_kernel_label(n4, p4, cus, shard=True), "ms_per_step": ms_s,
                                        "evals_per_s": n4 * p4 / (ms_s * 1e-3),
                                        "check": "bit-exact vs closed form" if ok_s else "MISMATCH"},
        "note": "one GPU holds the whole 100k-node table (75 KB of bit planes); the 8-GPU C4 run splits it "
                "(bench.py --mode nodeshard)"}
    ctx.close()
    return out


def host_cpu_share() -> int:
    """Host threads this process may use: its CPU affinity, capped by OMP_NUM_THREADS when the
    machine sets it (the GPU pool gives a one-GPU job a share of the host: 16 CPUs)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    env = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, min(n, int(env))) if env.isdigit() else n


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(unsched, node_digit, pod_digit, pod_tol, budget_s: float, mode: str, threads: int = 1):
    """The C restatement (oracle/msh_oracle.c) on this host's cores, on a bounded sample of the
    same workload: pods in chunks against the full node table until the budget is spent."""
    importlib.import_module("oracle.build").build_oracle()
    O = importlib.import_module("oracle.oracle")
    plugins = O.PluginSet(weights=[HEADLINE_WEIGHT], normalize=[HEADLINE_NORM])  # the headline list
    n = len(unsched)
    p = len(pod_digit)
    chunk = min(2000 * threads, p)
    done, t, pos = 0, 0.0, 0
    # cycle over the batch (wrapping) until the budget is spent: a 10-30 s sample
    while t < budget_s and p > 0:
        sl = slice(pos, min(pos + chunk, p))
        t0 = time.perf_counter()
        if mode == "sequential":
            O.c_schedule_sequential(unsched, node_digit, pod_digit[sl], pod_tol[sl], plugins)
        else:
            O.c_schedule_batch(unsched, node_digit, pod_digit[sl], pod_tol[sl], plugins, threads=threads)
        t += time.perf_counter() - t0
        done += sl.stop - sl.start
        pos = 0 if sl.stop >= p else sl.stop
    evals = float(n) * done
    return {"value": evals / t, "unit": "pod-node evals/s", "cores": threads, "kind": "port",
            "sample": f"{done} pods (cycling over the {p}-pod batch) x {n} nodes, C restatement "
                      f"({'scalar' if threads == 1 else f'OpenMP {threads} threads'}), {t:.2f} s",
            "cpu_model": cpu_model(), "host_cpus_visible": os.cpu_count(),
            "host_cpu_share": host_cpu_share(), "pods_per_s": done / t}


if __name__ == "__main__":
    main()
