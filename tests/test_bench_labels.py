"""bench.py names the kernel each measurement runs (it keys the PMC entries of profiles/r6_pmc_c3.json and the
rooflines by that name), restating the launchers' choices. These CPU tests keep the restatement in step
with the HIP sources: the thresholds bench.py copies, and the template-argument count of every kernel name
it builds against the kernel's declaration."""
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "mini-kube-scheduler_amd" / "csrc"


@pytest.fixture(scope="module")
def bench():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _const(src: str, name: str) -> int:
    m = re.search(rf"constexpr\s+int(?:32_t)?\s+{name}\s*=\s*(\d+)\s*;", src)
    assert m, f"{name} not found"
    return int(m.group(1))


def _template_arity(src: str, kernel: str) -> int:
    """Parameters of `template <...> __global__ ... kernel(` in the source."""
    m = re.search(rf"template\s*<([^>]*)>\s*__global__[^;{{]*?\b{kernel}\s*\(", src, re.S)
    assert m, f"{kernel} template not found"
    return len([p for p in m.group(1).split(",") if p.strip()])


def _label_arity(label: str) -> int:
    return len(label[label.index("<") + 1:label.rindex(">")].split(","))


def test_thresholds_match_the_launchers(bench):
    pair = (CSRC / "msh_pair.hip").read_text()
    assert bench.PAIR_LDS_MAX_GROUPS == _const(pair, "PAIR_LDS_MAX_GROUPS")
    assert bench.PAIR_LDS_BIG_GROUPS == _const(pair, "PAIR_LDS_BIG_GROUPS")
    assert bench.PAIR_SLICE_LDS_GROUPS == _const(pair, "PAIR_SLICE_LDS_GROUPS")
    internal = (CSRC / "msh_internal.h").read_text()
    assert _const(internal, "MULTI_MAX") == 32  # bench.py's multi-batch labels and PMC entries assume 32


@pytest.mark.parametrize("nodes,pods", [(1000, 10_000), (5000, 100_000), (40_000, 3000), (100_000, 1_000_000)])
def test_labels_have_the_kernels_template_arity(bench, nodes, pods):
    pair = (CSRC / "msh_pair.hip").read_text()
    seq = (CSRC / "msh_seq_kernel.h").read_text()
    cap = (CSRC / "msh_seq_cap.hip").read_text()
    arity = {"pair_kernel": _template_arity(pair, "pair_kernel"),
             "pair_lds_kernel": _template_arity(pair, "pair_lds_kernel"),
             "seq_kernel": _template_arity(seq, "seq_kernel"),
             "seq_capu_kernel": _template_arity(cap, "seq_capu_kernel")}
    labels = [bench.batch_kernel_label(nodes, pods, 256), bench.batch_kernel_label(nodes, pods, 256, kx=True),
              bench.batch_kernel_label(nodes, pods, 256, shard=True),
              bench.batch_kernel_label(nodes, pods, 256, multi=True, nb=32),
              bench.seq_kernel_label(min(nodes, 32_768)), bench.seq_kernel_label(min(nodes, 32_768), cap=True)]
    if nodes <= 32_768:
        labels.append(bench.seq_pair_label(nodes, pods, 256))
    for lab in labels:
        name = re.search(r"msh::(\w+)<", lab).group(1)
        assert _label_arity(lab) == arity[name], lab
