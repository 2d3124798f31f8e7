#!/usr/bin/env python3
"""Turn the rocprofv3 --pmc passes of tools/pmc_probe.py into profiles/pmc_traffic.json.

FETCH_SIZE / WRITE_SIZE (KiB per dispatch) are calibrated on this repo's own access pattern,
as MI355X_MICROARCH.md's HBM section prescribes for non-16-B accesses:
  read factor  = known bytes read by oc_checksum_kernel (num_planes x pitch, dword loads)
                 / (FETCH_SIZE x 1024)
  write factor = known bytes written by oc_reset_kernel (num_planes x pitch, dword stores)
                 / (WRITE_SIZE x 1024)
HBM traffic of a step launch = FETCH x read factor + WRITE x write factor (mean over launches,
the first launch of each kernel dropped).

usage: pmc_report.py FETCH_DIR WRITE_DIR OUT.json
"""
import csv
import glob
import json
import os
import sys

B, NP, A = 1 << 20, 17, 2  # tools/pmc_probe.py workload
PITCH = B
NFUSED = (20, 100)  # tools/pmc_probe.py: 3 oc_step_n dispatches of each, in this order


def per_kernel(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit("no counter_collection.csv under %s" % d)
    out = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                name = row["Kernel_Name"]
                key = next((k for k in ("oc_step_n_kernel", "oc_step_kernel", "oc_checksum_kernel", "oc_reset_kernel")
                            if k in name), None)
                if key:
                    out.setdefault(key, []).append((int(row.get("Dispatch_Id", 0)), float(row["Counter_Value"])))
    return {k: [v for _, v in sorted(vs)] for k, vs in out.items()}


def mean_tail(v):
    v = v[1:] if len(v) > 1 else v
    return sum(v) / len(v)


def main():
    fdir, wdir, out = sys.argv[1:4]
    fetch, write = per_kernel(fdir, "FETCH_SIZE"), per_kernel(wdir, "WRITE_SIZE")
    known = NP * PITCH
    rf = known / (mean_tail(fetch["oc_checksum_kernel"]) * 1024)
    wf = known / (mean_tail(write["oc_reset_kernel"]) * 1024)
    res = {"workload": "partial-divider_salad, 2 agents, 2^20 envs (tools/pmc_probe.py)",
           "read_factor": rf, "write_factor": wf,
           "raw_kib": {k: {"FETCH_SIZE": mean_tail(fetch.get(k, [0])), "WRITE_SIZE": mean_tail(write.get(k, [0]))}
                       for k in sorted(set(fetch) | set(write))}}
    f_step, w_step = mean_tail(fetch["oc_step_kernel"]) * 1024 * rf, mean_tail(write["oc_step_kernel"]) * 1024 * wf
    alg = (2 * NP + 2 * A + 1) * B
    res["oc_step_kernel"] = {"read_bytes": f_step, "write_bytes": w_step, "hbm_bytes_per_launch": f_step + w_step,
                             "algorithmic_bytes_per_launch": alg, "ratio": (f_step + w_step) / alg}
    if "oc_step_n_kernel" in fetch:
        shapes = {}
        for i, n in enumerate(NFUSED):
            fv, wv = fetch["oc_step_n_kernel"][3 * i:3 * i + 3], write["oc_step_n_kernel"][3 * i:3 * i + 3]
            fn, wn = mean_tail(fv) * 1024 * rf, mean_tail(wv) * 1024 * wf
            algn = (NP + n * (NP + 2 * A + 1)) * B
            shapes[str(n)] = {"steps_per_launch": n, "read_bytes": fn, "write_bytes": wn,
                              "hbm_bytes_per_launch": fn + wn, "algorithmic_bytes_per_launch": algn,
                              "ratio": (fn + wn) / algn}
        res["oc_step_n_kernel"] = {"by_steps_per_launch": shapes}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
