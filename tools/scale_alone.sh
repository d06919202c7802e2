#!/bin/bash
# Strong-scaling prediction on one GPU: every rank's shard of N routed ALONE with the full bench step
# of the workload (C3: parameter network, fused daily objective, backward, optimizer).
# Usage: bash tools/scale_alone.sh WL "1 2 4 8" [bench args]  -> gpurun_out/scale_WL/*.json + summary
WL=${1:-c3}; NS=${2:-"1 2 4 8"}; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/scale_$WL
mkdir -p $OUT
for N in $NS; do
  for ((r = 0; r < N; r++)); do
    WORLD_SIZE=$N RANK=$r LOCAL_RANK=0 DDR_BENCH_ALONE=1 timeout -k 10 300 python3 $R/bench.py --workload $WL \
      --steps 3 --warmup 1 --no-cpu-baseline --dropin-steps 0 "$@" > $OUT/n${N}_r$r.json 2> $OUT/n${N}_r$r.err \
      || { echo "N=$N rank $r failed"; tail -3 $OUT/n${N}_r$r.err; exit 1; }
  done
done
python3 - "$OUT" $NS <<'PY'
import json, sys, glob
out, Ns = sys.argv[1], [int(a) for a in sys.argv[2:]]
res = {}
for N in Ns:
    ranks = [json.loads(open(f"{out}/n{N}_r{r}.json").read().strip().splitlines()[-1]) for r in range(N)]
    ms = [d["ms_per_step"] for d in ranks]
    res[N] = {"ms_max": max(ms), "ranks": [{"rank": r, "reaches": d["config"]["reaches"], "ms": d["ms_per_step"],
                                             "kernels": {k: round(v["kernel_ms"], 2) for k, v in d["kernels"].items()}}
                                            for r, d in enumerate(ranks)]}
base = res[Ns[0]]["ms_max"] * Ns[0]
for N in Ns:
    res[N]["speedup"] = base / res[N]["ms_max"] / Ns[0] * Ns[0] if Ns[0] == 1 else None
    print(N, round(res[N]["ms_max"], 2), res[N]["speedup"] and round(res[N]["speedup"], 2))
json.dump(res, open(f"{out}/summary.json", "w"))
PY
