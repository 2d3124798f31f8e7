# Round 5 pass E: A/B of the C5 kernels over four builds (one box, alternating processes):
# round 4's node table, the hybrid table, + branch-free row code, + side-split Merge walk.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r5e}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python tools/bounds_ab.py --libs tools/ab_libs/lib_nodetable.so tools/ab_libs/lib_hybrid.so \
  tools/ab_libs/lib_bfree.so tools/ab_libs/lib_side.so --rounds 3 > $O/ab.jsonl 2> $O/ab.err || { echo AB_FAILED; tail -20 $O/ab.err; exit 1; }
python - <<PY
import json, collections
rows = [json.loads(l) for l in open("$O/ab.jsonl")]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    for k, v in r.items():
        if k.endswith("_ms"):
            agg[r["lib"]][k].append(v * 1e3)
for lib, d in agg.items():
    print(lib, " ".join("%s %.1f-%.1f" % (k[:-3], min(v), max(v)) for k, v in d.items()), {r["digest"] for r in rows if r["lib"] == lib})
PY
