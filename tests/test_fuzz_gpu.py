"""Randomised GPU parity sweep: a bounded sweep in every GPU run (BOUNDED_CASES cases of at most
BOUNDED_PAIRS (pod, node) pairs each, a seed base of its own), and the long opt-in sweep (MSH_FUZZ=<cases>).

Each case draws a table size, a pod count, the filter / prescore lists, a score list of NodeNumber and up to
three score-column plugins with random weights and NormalizeScore modes, columns of random range (small,
signed, the whole int32 range, constant) and random unschedulable / tolerates / no-digit rates, then runs
the batch entry point, then patches random nodes (msh_patch_nodes) and runs the multi-batch device
entry point on 1-5 slices of the pods, then the node-sharded path over 2-4 shards at random bounds
(merged in-process as the collectives would), and, for lists without score columns, the sequential one
with and without a capacity, against the oracle (oracle/msh_oracle.c, the restatement of minisched/minisched.go:115-199,
304-325): idx / score / status bit-exact, and the sequential node counts. The summary (cases per
category, any mismatch with its seed) goes to $MSH_FUZZ_OUT (default gpurun_out/fuzz_summary.json).
"""
from __future__ import annotations

import json
import os
import time
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CASES = int(os.environ.get("MSH_FUZZ", "0"))
COLS = ["ScoreColumn0", "ScoreColumn1", "ScoreColumn2", "ScoreColumn3"]
WEIGHTS = [1, 2, 3, 7, 100, 1 << 16, 1 << 32]


BOUNDED_CASES = 500
BOUNDED_PAIRS = 2e7


def _case(rng, max_pairs=1.5e8):
    n = int(np.exp(rng.uniform(0, np.log(60_000))))
    p = int(np.exp(rng.uniform(0, np.log(30_000))))
    while n * p > max_pairs:
        p //= 2
    p = max(p, 1)
    unsched = (rng.random(n) < rng.choice([0.0, 0.1, 0.5, 1.0])).astype(np.uint8)
    nd = rng.integers(0, 10, n).astype(np.int8)
    nd[rng.random(n) < rng.choice([0.0, 0.1, 1.0])] = -1
    pd = rng.integers(0, 10, p).astype(np.int8)
    pd[rng.random(p) < rng.choice([0.0, 0.1, 1.0])] = -1
    pt = (rng.random(p) < rng.choice([0.0, 0.05, 0.5, 1.0])).astype(np.uint8)
    filters = ["NodeUnschedulable"] if rng.random() < 0.8 else []
    prescore = ["NodeNumber"] if rng.random() < 0.8 else []
    pool = ["NodeNumber"] + list(rng.choice(COLS, size=int(rng.integers(0, 4)), replace=False))
    score = [s for s in rng.permutation(pool) if s != "NodeNumber" or rng.random() < 0.85]
    weights = [int(rng.choice(WEIGHTS)) for _ in score]
    norms = [int(rng.integers(0, 4)) for _ in score]
    cols = {}
    for k in range(4):
        kind = rng.integers(0, 4)
        if kind == 0:
            cols[k] = rng.integers(0, 101, n)
        elif kind == 1:
            cols[k] = rng.integers(-50, 51, n)
        elif kind == 2:
            cols[k] = rng.integers(-(1 << 31), (1 << 31) + 1, n)
        else:
            cols[k] = np.full(n, int(rng.integers(-5, 6)))
    return n, p, unsched, nd, pd, pt, filters, prescore, score, weights, norms, cols


def test_fuzz_parity_bounded(msh, oracle):
    """The bounded sweep of every GPU run: fixed seeds 20261100.., cases small enough for well under a minute (120 cases: 1 s on MI355X)."""
    _sweep(msh, oracle, BOUNDED_CASES, 20261100, BOUNDED_PAIRS, Path("gpurun_out/fuzz_bounded_summary.json"))


@pytest.mark.skipif(CASES <= 0, reason="opt-in sweep: set MSH_FUZZ=<cases>")
def test_fuzz_parity(msh, oracle):
    _sweep(msh, oracle, CASES, int(os.environ.get("MSH_FUZZ_SEED", "20261018")), 1.5e8,
           Path(os.environ.get("MSH_FUZZ_OUT", "gpurun_out/fuzz_summary.json")))


def _sweep(msh, oracle, CASES, seed0, max_pairs, out):
    out.parent.mkdir(parents=True, exist_ok=True)
    torch = pytest.importorskip("torch")
    stats = {"batch": 0, "batch_w_columns": 0, "patch_then_multi_batch": 0, "node_sharded": 0, "sequential": 0,
             "sequential_capacity": 0, "pairs": 0}
    fails = []
    t0 = time.time()
    with msh.DeviceContext(0) as ctx:
        for c in range(CASES):
            seed = seed0 + c
            rng = np.random.default_rng(seed)
            n, p, u, nd, pd, pt, fl, pre, sc, w, nm, cols = _case(rng, max_pairs)
            ps = oracle.PluginSet(filters=fl, prescore=pre, score=sc, weights=w, normalize=nm)
            ctx.set_plugins(fl, pre, [msh.ScorePluginConfig(s, ww, msh.Normalize(m)) for s, ww, m in zip(sc, w, nm)])
            ctx.upload_nodes(u, nd)
            has_cols = any(s in COLS for s in sc)
            for k in range(4):
                if COLS[k] in sc:
                    ctx.upload_score_column(COLS[k], cols[k])
            got = ctx.schedule_batch(pd, pt)
            want = oracle.c_schedule_batch(u, nd, pd, pt, ps, threads=16, cols=cols)
            stats["batch_w_columns" if has_cols else "batch"] += 1
            stats["pairs"] += n * p
            desc = {"seed": seed, "n": n, "p": p, "filters": fl, "prescore": pre, "score": sc, "weights": w,
                    "normalize": nm}
            if not all((g == x).all() for g, x in zip(got, want[:3])):
                fails.append(dict(desc, mode="batch"))
            # a patch of random nodes (a cordon flip / digit change: msh_patch_nodes, inline or scattered),
            # then the multi-batch device entry point on 1-5 slices of the pods
            k = int(min(n, rng.choice([1, 5, 64, 65, 2000])))
            pidx = rng.choice(n, size=k, replace=False).astype(np.int32)
            u2, nd2 = u.copy(), nd.copy()
            u2[pidx] = rng.integers(0, 2, k)
            nd2[pidx] = rng.integers(-1, 10, k)
            ctx.patch_nodes(pidx, u2[pidx], nd2[pidx])
            cuts = np.unique(np.concatenate([[0, p], rng.integers(0, p + 1, int(rng.integers(0, 5)))]))
            dev = torch.device("cuda:0")
            bufs = [[torch.from_numpy(pd[x:y]).to(dev), torch.from_numpy(pt[x:y]).to(dev),
                     torch.full((y - x,), -7, dtype=torch.int32, device=dev),
                     torch.full((y - x,), -7, dtype=torch.int64, device=dev),
                     torch.full((y - x,), -7, dtype=torch.int32, device=dev)] for x, y in zip(cuts, cuts[1:])]
            descs = ctx.batch_descs([(len(b[0]), *[t.data_ptr() for t in b]) for b in bufs])
            ctx.schedule_batches_device(descs, stream=torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            got = tuple(np.concatenate([b[i].cpu().numpy() for b in bufs]) for i in (2, 3, 4))
            want = oracle.c_schedule_batch(u2, nd2, pd, pt, ps, threads=16, cols=cols)
            stats["patch_then_multi_batch"] += 1
            if not all((g == x).all() for g, x in zip(got, want[:3])):
                fails.append(dict(desc, mode="patch+multi", patched=k, batches=len(bufs)))
            u, nd = u2, nd2
            # the node-sharded path on 2-4 shards at random List-order bounds, merged here as the
            # collectives would (MAX / MIN over the shards' device buffers): the reference lists through
            # msh_shard_keys_device + msh_decode_keys_device, score-column lists through msh_generic_*
            if n >= 4:
                nsh = int(rng.integers(2, 5))
                bounds = [0] + sorted(int(x) for x in rng.choice(np.arange(1, n), size=nsh - 1, replace=False)) + [n]
                d_pd, d_pt = torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev)
                shards = []
                for lo, hi in zip(bounds, bounds[1:]):
                    c2 = msh.DeviceContext(0)
                    c2.set_plugins(fl, pre, [msh.ScorePluginConfig(s_, ww, msh.Normalize(m)) for s_, ww, m in zip(sc, w, nm)])
                    c2.upload_nodes(u[lo:hi], nd[lo:hi])
                    for kk in range(4):
                        if COLS[kk] in sc:
                            c2.upload_score_column(COLS[kk], cols[kk][lo:hi])
                    shards.append((c2, lo))
                hs = torch.cuda.current_stream().cuda_stream
                oi = torch.empty(p, dtype=torch.int32, device=dev)
                osc = torch.empty(p, dtype=torch.int64, device=dev)
                ost = torch.empty(p, dtype=torch.int32, device=dev)
                if not has_cols:
                    merged = None
                    for c2, lo in shards:
                        keys = torch.empty(c2.shard_keys_len(p), dtype=torch.int32, device=dev)
                        c2.shard_keys_device(p, d_pd.data_ptr(), d_pt.data_ptr(), lo, keys.data_ptr(), hs)
                        merged = keys if merged is None else torch.maximum(merged, keys)
                    shards[0][0].decode_keys_device(p, d_pd.data_ptr(), d_pt.data_ptr(), merged.data_ptr(),
                                                    oi.data_ptr(), osc.data_ptr(), ost.data_ptr(), hs)
                else:
                    n_ext = shards[0][0].generic_ext_len(p)
                    ext = None
                    if n_ext:
                        exts = []
                        for c2, lo in shards:
                            e_ = torch.empty(n_ext, dtype=torch.int64, device=dev)
                            c2.generic_extents_device(p, d_pd.data_ptr(), d_pt.data_ptr(), e_.data_ptr(), hs)
                            exts.append(e_)
                        ext = torch.stack(exts).max(dim=0).values.contiguous()
                    tots, idxs = [], []
                    for c2, lo in shards:
                        t_ = torch.empty(p, dtype=torch.int64, device=dev)
                        i_ = torch.empty(p, dtype=torch.int32, device=dev)
                        c2.generic_best_device(p, d_pd.data_ptr(), d_pt.data_ptr(), ext.data_ptr() if ext is not None else 0,
                                               lo, t_.data_ptr(), i_.data_ptr(), hs)
                        tots.append(t_)
                        idxs.append(i_)
                    mt = torch.stack(tots).max(dim=0).values.contiguous()
                    for (c2, lo), t_, i_ in zip(shards, tots, idxs):
                        c2.generic_candidates_device(p, t_.data_ptr(), mt.data_ptr(), i_.data_ptr(), hs)
                    mi = torch.stack(idxs).min(dim=0).values.contiguous()
                    shards[0][0].generic_decode_device(p, d_pd.data_ptr(), mt.data_ptr(), mi.data_ptr(), oi.data_ptr(),
                                                       osc.data_ptr(), ost.data_ptr(), hs)
                torch.cuda.synchronize()
                got = (oi.cpu().numpy(), osc.cpu().numpy(), ost.cpu().numpy())
                stats["node_sharded"] += 1
                if not all((g == x).all() for g, x in zip(got, want[:3])):
                    fails.append(dict(desc, mode="node-sharded", bounds=bounds))
                for c2, _ in shards:
                    c2.close()
            if not has_cols:
                cap = int(rng.choice([0, 0, 1, 3]))
                ctx.reset_node_pod_counts()
                got = ctx.schedule_sequential(pd, pt, cap)
                want = oracle.c_schedule_sequential(u, nd, pd, pt, ps, cap)
                stats["sequential_capacity" if cap else "sequential"] += 1
                if not (all((g == x).all() for g, x in zip(got, want[:3]))
                        and (ctx.node_pod_counts() == want[3]).all()):
                    fails.append(dict(desc, mode="sequential", capacity=cap))
            if (c + 1) % 25 == 0:  # progress to a file too: pytest holds the test's stdout until it ends
                line = f"fuzz: {c + 1}/{CASES} cases, {len(fails)} mismatches, {time.time() - t0:.0f} s"
                print(line, flush=True)
                out.with_suffix(".progress").write_text(line + "\n")
    summary = {"cases": CASES, "seed0": seed0, "counts": stats, "mismatches": fails,
               "seconds": round(time.time() - t0, 1)}
    out.write_text(json.dumps(summary, indent=1))
    assert not fails, fails[:3]
