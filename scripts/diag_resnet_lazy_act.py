import os, sys, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import pgdist
from pgdist.models import build_model
from pgdist.engine.native_step import NativeTrainStep
from pgdist.engine.resnet_executor import ResNet50Executor
dev = torch.device("cuda", 0)
stem = sys.argv[1]
ResNet50Executor.STEM = stem
src = torch.randint(0, 256, (16, 64, 64, 3), dtype=torch.uint8, device=dev, generator=torch.Generator(device=dev).manual_seed(5))
labels = torch.arange(16, device=dev) % 10
for fold in (128, 0):
    ResNet50Executor.FOLD_MAX_CIN = fold
    for lazy in ("0", "act", "0", "act", "1"):
        os.environ["PGDIST_BN_LAZY"] = lazy
        torch.manual_seed(0)
        st = NativeTrainStep(build_model("resnet50", num_classes=10), 8, dev, img_size=64, lr=1e-3, use_graph=False)
        st.set_data(src, labels)
        losses = []
        for i in range(4):
            st.run((torch.arange(8, device=dev) + 3 * i) % 16)
            l, _, n = st.read_metrics()
            losses.append(round(l / n, 4))
        print("fold", fold, "lazy", lazy, losses, flush=True)
