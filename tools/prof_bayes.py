#!/usr/bin/env python3
"""cProfile of bench.py's bayes line (256 delegators' Level-1 belief updates in one
bayes_update_batch call on the C5 layout) on the GPU box: where the host time goes.
Writes gpurun_out/<tag>/bayes_prof.txt."""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gym-cooking_amd"))

import torch  # noqa: E402

import bench  # noqa: E402

out = sys.argv[1]
os.makedirs(out, exist_ok=True)
dev = torch.device("cuda", 0)
bench.measure_bayes(dev, 1, n_updates=32, n_seq=1)  # warm-up: library, tables, allocator
pr = cProfile.Profile()
pr.enable()
r = bench.measure_bayes(dev, 1, n_updates=256, n_seq=1)
pr.disable()
with open(os.path.join(out, "bayes_prof.txt"), "w") as f:
    f.write("%s\n" % {k: v for k, v in r.items() if not isinstance(v, (dict, list))})
    st = pstats.Stats(pr, stream=f)
    st.sort_stats("tottime").print_stats(40)
    st.sort_stats("cumulative").print_stats(40)
print("done")
