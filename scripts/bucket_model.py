"""The gradient-bucket layout the reducer's objective picks for MobileNetV2 under an xGMI
all-reduce cost model (CPU only; parallel/ddp.py candidate_layouts / choose_layout).

On a real node the reducer measures the all-reduce times and the ready times itself (second
warm-up step).  A one-GPU rehearsal cannot: 8 processes time-share one GPU, so every collective
measures ~30 ms and the objective rightly picks the fewest buckets.  This prints the layout for
plausible 8-GPU numbers instead: all-reduce t(n) = alpha + bytes / bw, a 2.3 ms backward
(the bs128 step's backward on one MI355X), gradient ready times from the layer-size model.

    python scripts/bucket_model.py [--alpha-us 25] [--gbps 60] [--t-bwd-us 2300]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pgdist  # noqa: E402,F401


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--alpha-us", type=float, default=25.0)
    ap.add_argument("--gbps", type=float, default=60.0)
    ap.add_argument("--t-bwd-us", type=float, default=2300.0)
    a = ap.parse_args()
    from pgdist.engine.flat import FlatParams
    from pgdist.models import mobilenet_v2
    from pgdist.parallel.ddp import build_buckets, candidate_layouts, choose_layout, estimate_ready_times, \
        simulate_buckets
    torch.manual_seed(0)
    model = mobilenet_v2(10)
    flat = FlatParams(model, torch.device("cpu"))
    ranges = [(nm,) + flat.range_of(nm) for nm in flat.order]
    ready = estimate_ready_times(model, 224, a.t_bwd_us)
    t_ar = lambda n: a.alpha_us + n * 4 / (a.gbps * 1e3)   # noqa: E731  (us)
    cands = candidate_layouts(ranges, 1.0, flat.numel * 4 / 2 ** 20)
    cost, key = choose_layout(cands, ready, a.t_bwd_us, t_ar)
    best = cands[key]
    print(f"cost model: all-reduce {a.alpha_us} us + bytes / {a.gbps} GB/s; backward {a.t_bwd_us} us; "
          f"gradient {flat.numel * 4 / 2 ** 20:.2f} MiB")
    print(f"chosen cap / last cap (MiB): {key[0]} / {key[1]}; simulated exposed {cost[key]:.1f} us")
    for s, e, names in best:
        r = max(ready[n] for n in names)
        print(f"  bucket {(e - s) * 4 / 2 ** 20:6.2f} MiB  {len(names):3d} tensors  ready at {r:7.1f} us")
    old = build_buckets(ranges, 8 << 20, 1 << 20)
    print(f"round-4 objective's pick (8 MiB cap, no tail bucket): {len(old)} buckets "
          f"{[round((e - s) * 4 / 2 ** 20, 2) for s, e, _ in old]} MiB, simulated exposed "
          f"{simulate_buckets(old, ready, a.t_bwd_us, t_ar):.1f} us")


if __name__ == "__main__":
    main()
