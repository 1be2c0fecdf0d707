"""Print the e2e block and the K=20 values of a bench re-check (gpurun_out/b2)."""
import json

d = json.load(open("gpurun_out/b2/bench.json"))
print(json.dumps(d["e2e"])[:1600])
for f in ("k20a", "k20b"):
    d = json.load(open("gpurun_out/b2/" + f + ".json"))
    print(f, d["value"], d["ms_per_step"] * 1e3)
