"""Phase anatomy of the sequential-commit kernel (diagnostic -DMSH_STAMPS build only).

Per wave, cycles (s_memtime, shader clock) summed over the pods: 0 = pod fetch + scan,
1 = wave reductions, 2 = LDS write + barrier, 3 = final cross-wave reduction (wave 0, or every
wave with a capacity), 4 unused, 5 = decode + output + commit + loop (measured at the next pod's
top). Prints cycles per pod per phase for each wave.
"""
import ctypes as C
import importlib
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
build = importlib.import_module("mini-kube-scheduler_amd.build")
os.environ["MSH_LIBRARY"] = str(build.build_diagnostic())
import torch  # noqa: E402
msh = importlib.import_module("mini-kube-scheduler_amd")
msh._native.LIB_PATH = Path(os.environ["MSH_LIBRARY"])
synth = importlib.import_module("mini-kube-scheduler_amd.synthetic")
lib = msh._native.lib()
lib.msh_debug_read_stamps.argtypes = [C.c_void_p, C.c_int]
lib.msh_debug_clear_stamps.argtypes = []
n, p = 5000, 20000
ctx = msh.DeviceContext(0)
u, nd, pd, pt = synth.make_soa(n, p)
ctx.upload_nodes(u, nd)
dev = torch.device("cuda:0")
d_pd, d_pt = torch.from_numpy(pd).to(dev), torch.from_numpy(pt).to(dev)
oi = torch.empty(p, dtype=torch.int32, device=dev)
osc = torch.empty(p, dtype=torch.int64, device=dev)
ost = torch.empty(p, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream()
for waves in os.environ.get("WAVES", "8,16").split(","):
    for cap in (0, 1000):
        os.environ["MSH_SEQ_WAVES"] = waves
        assert lib.msh_debug_clear_stamps() == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        ctx.schedule_sequential_device(p, d_pd.data_ptr(), d_pt.data_ptr(), cap, oi.data_ptr(), osc.data_ptr(),
                                       ost.data_ptr(), s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
        ctx.reset_node_pod_counts() if hasattr(ctx, "reset_node_pod_counts") else None
        buf = np.zeros(16 * 8 * 2, np.uint64)
        assert lib.msh_debug_read_stamps(buf.ctypes.data, 16) == 0
        st = buf[:16 * 8].reshape(16, 8).astype(np.float64)
        rows = {int(w): [round(x / p, 1) for x in st[w, :6]] for w in range(16) if st[w, 6] > 0}
        print(json.dumps({"waves": waves, "cap": cap, "us_per_pod": e0.elapsed_time(e1) * 1e3 / p,
                          "cycles_per_pod_by_phase[scan,reduce,lds+barrier,final,-,decode+commit+loop]": rows}))
