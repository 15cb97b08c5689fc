"""Per-parameter gradient differences of one MobileNetV2 step: lazy vs launch BN finalize
(and launch vs launch for the float-atomic noise floor)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pgdist  # noqa: F401,E402
from pgdist.models import mobilenet_v2  # noqa: E402
from pgdist.engine.native_step import NativeTrainStep  # noqa: E402

dev = torch.device("cuda", 0)
src = torch.randint(0, 256, (32, 32, 32, 3), dtype=torch.uint8, device=dev,
                    generator=torch.Generator(device=dev).manual_seed(7))
labels = torch.randint(0, 10, (32,), device=dev, generator=torch.Generator(device=dev).manual_seed(8))
B = int(os.environ.get("DIAG_B", "16"))
S = int(os.environ.get("DIAG_S", "96"))
res = {}
for tag, lazy in (("lazy", "1"), ("launch", "0"), ("launch2", "0")):
    os.environ["PGDIST_BN_LAZY"] = lazy
    torch.manual_seed(100)
    st = NativeTrainStep(mobilenet_v2(10), B, dev, img_size=S, lr=1e-3, use_graph=False, train_augment=False)
    st.set_data(src, labels)
    st.run(torch.arange(B, device=dev) % 32)
    torch.cuda.synchronize()
    g = {n: st.flat.grad[slice(*st.flat.range_of(n))].clone() for n in st.flat.order}
    res[tag] = (g, st.read_metrics()[0])
    print(tag, "loss", res[tag][1], "gnorm", st.flat.grad.norm().item(), flush=True)
for a, b in (("lazy", "launch"), ("launch2", "launch")):
    ga, gb = res[a][0], res[b][0]
    rows = []
    for n in gb:
        d = (ga[n] - gb[n]).norm().item()
        r = d / (gb[n].norm().item() + 1e-20)
        rows.append((r, n, gb[n].norm().item()))
    rows.sort(reverse=True)
    print(f"--- {a} vs {b}: worst relative gradient differences")
    for r, n, nm in rows[:12]:
        print(f"  {r:9.3e}  {n}  (|g|={nm:.3e})")
    order = list(gb)
    print("  in backward-completion order (first 8 / last 8):")
    for n in order[:8] + order[-8:]:
        print(f"    {(ga[n] - gb[n]).norm().item() / (gb[n].norm().item() + 1e-20):9.3e}  {n}")
