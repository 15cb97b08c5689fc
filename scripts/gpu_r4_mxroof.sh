#!/bin/bash
# Round 4: per-op isolated times of the bs512 fp8 step with the fp8 tile GEMMs on the
# 16x16x128 block-scaled MFMA (MX=1) vs the 16x16x32 fp8 MFMA (MX=0)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/mxr && export TMPDIR=/tmp
O=gpurun_out/mxr
for e in 1 0; do
  PGDIST_F8_MX=$e timeout -k 10 400 python -u scripts/roofline.py --batch 512 --fp8 1 --iters 10 --out $O/roof_mx$e.txt > $O/roof_mx$e.log 2>&1 || { tail -20 $O/roof_mx$e.log; exit 1; }
done
python - <<'PY'
import re
def load(p):
    d = {}
    for ln in open(p):
        f = ln.split()
        if len(f) > 6 and f[0].isdigit() and f[2] == "pw_gemm":
            d[int(f[0])] = (float(f[3]), " ".join(f[8:]))
    return d
a, b = load("gpurun_out/mxr/roof_mx1.txt"), load("gpurun_out/mxr/roof_mx0.txt")
tot1 = tot0 = 0
for k in sorted(a):
    if k in b and abs(a[k][0] - b[k][0]) > 0.5:
        print(f"{k:4d} mx1 {a[k][0]:7.1f} mx0 {b[k][0]:7.1f}  {a[k][1]}")
    tot1 += a[k][0]; tot0 += b.get(k, (0,))[0]
print(f"pw_gemm total mx1 {tot1:.1f} us  mx0 {tot0:.1f} us")
PY
