"""Host-side enqueue cost of one native training step vs its wall time.

If enqueue ms/step approaches wall ms/step the GPU is starved by the Python launch path."""
import sys
import time

import torch

sys.path.insert(0, '.')
import pgdist  # noqa: F401,E402
from pgdist.engine.native_step import NativeTrainStep  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "mobilenet_v2"
graph = int(sys.argv[2]) if len(sys.argv) > 2 else 0
dev = torch.device('cuda', 0)
st = NativeTrainStep.for_benchmark(model, 128, dev, use_graph=bool(graph))
for _ in range(5):
    st.bench_step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    st.bench_step()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"{model} graph={graph}: host enqueue {1e3 * (t1 - t0) / 20:.2f} ms/step, wall {1e3 * (t2 - t0) / 20:.2f} ms/step")
