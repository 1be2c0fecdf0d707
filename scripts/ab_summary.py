import json,collections,sys
d=collections.defaultdict(list)
for l in open(sys.argv[1]):
    j=json.loads(l); d[(j["tag"],j["batches_per_launch"])].append(round(j["us_per_batch"],3))
for k,v in sorted(d.items()): print(k,v)
