import time, torch, sys
sys.path.insert(0, '.')
import pgdist
from pgdist.engine.native_step import NativeTrainStep
dev = torch.device('cuda', 0)
st = NativeTrainStep.for_benchmark('mobilenet_v2', 128, dev, use_graph=False)
for _ in range(5): st.bench_step()
torch.cuda.synchronize()
# host cost: enqueue 20 steps, measure host time until return (GPU queue absorbs)
t0 = time.perf_counter()
for _ in range(20): st.bench_step()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"host enqueue {1e3*(t1-t0)/20:.2f} ms/step, wall {1e3*(t2-t0)/20:.2f} ms/step")
