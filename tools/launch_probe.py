#!/usr/bin/env python3
"""Host time of the headline's launch call (the bound oc_step_n launcher, bench.py's driver
shape), on an idle queue (synchronize before each call, as the bench's window starts) and on a
busy one (back to back), on torch's default stream and on a created (non-default) stream, and
again after the bench's world-1 RCCL group and communicator are up (dist.init).
Prints one JSON line: microsecond percentiles per case."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-cooking_amd")]
import torch  # noqa: E402
from gym_cooking_amd.engine import OvercookedBatch  # noqa: E402


def main():
    dev = "cuda:0"
    if "--spin" in sys.argv:  # as bench.py --host-wait spin: hipDeviceScheduleSpin before torch touches the device
        import ctypes
        hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
        assert hip.hipSetDevice(ctypes.c_int(0)) == 0 and hip.hipSetDeviceFlags(ctypes.c_uint(1)) == 0
    B, A, n = 1 << 20, 2, 20
    out = {}
    cases = [("default", False), ("created", False), ("default", True)]
    for sname, with_rccl in cases:
        if with_rccl:  # the bench's world-1 RCCL group and direct communicator (dist.init)
            from gym_cooking_amd import dist as ocdist
            ocdist.init("nccl")
        st = torch.cuda.current_stream(dev) if sname == "default" else torch.cuda.Stream(device=dev)
        with torch.cuda.stream(st):
            eb = OvercookedBatch("partial-divider_salad", A, B, max_T=100, device=dev)
            s = eb.new_state()
            eb.reset(s)
            S = s.numel()
            acts = eb.new_actions(n)
            for t in range(n):
                eb.gen_actions(acts[t], t, 7)
            traj = torch.empty(n * S, dtype=torch.uint8, device=dev)
            ex = torch.empty(n * A * eb.pitch, dtype=torch.uint8, device=dev)
            coll = torch.empty(n * eb.pitch, dtype=torch.uint8, device=dev)
            stats = eb.new_stats()
            tot = torch.zeros(5, dtype=torch.int64, device=dev)
            f = eb.step_n_launcher(s, traj[(n - 1) * S:], acts.reshape(-1), n, traj, ex, coll, stats, tot)
            for _ in range(5):
                f()
            torch.cuda.synchronize()
            idle, busy = [], []
            for _ in range(60):
                torch.cuda.synchronize()
                t0 = time.perf_counter_ns()
                f()
                idle.append((time.perf_counter_ns() - t0) / 1e3)
            torch.cuda.synchronize()
            for _ in range(60):
                t0 = time.perf_counter_ns()
                f()
                busy.append((time.perf_counter_ns() - t0) / 1e3)
            torch.cuda.synchronize()
            # the first call of a freshly bound launcher (the bench binds its window's launchers
            # ahead and calls them for the first time inside the window)
            first = []
            for _ in range(20):
                g = eb.step_n_launcher(s, traj[(n - 1) * S:], acts.reshape(-1), n, traj, ex, coll, stats, tot)
                torch.cuda.synchronize()
                t0 = time.perf_counter_ns()
                g()
                first.append((time.perf_counter_ns() - t0) / 1e3)
            torch.cuda.synchronize()
        q = lambda v: {p: round(sorted(v)[int(p / 100 * (len(v) - 1))], 1) for p in (10, 50, 90)}  # noqa: E731
        out[sname + ("+rccl" if with_rccl else "")] = {"idle_us": q(idle), "busy_us": q(busy), "first_call_us": q(first)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
