import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
for r in rows:
    print(r["N"], r["depth"], r["rpw"], r.get("rpw_used", ""), r.get("variant", ""), round(r["wall_gcups"]),
          round(r["kernel_gcups"]), round(r["launch_ms"], 4))
best = {}
for r in rows:
    if r["wall_gcups"] > best.get(r["N"], {"wall_gcups": 0})["wall_gcups"]:
        best[r["N"]] = r
for n, r in best.items():
    print("best", n, r["depth"], r["rpw"], r.get("rpw_used"), r.get("variant"), round(r["wall_gcups"]))
