# Round 5 pass G: A/B of the C5 kernels (round 4's build, the device-memory-distance restore, +
# the xy table and 24-bit multiplies) and of the C3 step kernel (launch bounds 5 vs 6 waves).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r5g}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python tools/bounds_ab.py --libs tools/ab_libs/lib_nodetable.so tools/ab_libs/lib_gd.so \
  tools/ab_libs/lib_xy.so --rounds 3 > $O/ab.jsonl 2> $O/ab.err || { echo AB_FAILED; tail -20 $O/ab.err; exit 1; }
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
timeout -k 10 900 python tools/step_ab.py --libs tools/ab_libs/lib_xy.so tools/ab_libs/lib_xylb6.so --rounds 3 > $O/step_ab.jsonl 2> $O/step_ab.err || { echo STEP_AB_FAILED; tail -20 $O/step_ab.err; exit 1; }
cat $O/step_ab.jsonl
