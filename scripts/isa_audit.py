"""ISA audit of hipcc's s_waitcnt placement in loops (gfx950).

gfx950 counts loads and stores in one vmcnt queue; hipcc's waitcnt pass waits vmcnt(0) where
paths with different loads in flight join, where a builtin LDS DMA may alias a later LDS read,
or where a load it still counts as pending is first used inside a loop.  Each of these
serialises a software pipeline (docs/PERF_NOTES.md round 5).  This compiles a kernel source to
gfx950 assembly and lists, per kernel and loop, the COMPILER-inserted vmcnt waits inside the
loop body (inline-asm waits are the kernels' own counted waits and are not listed).

    python scripts/isa_audit.py csrc/kernels/dwconv.hip [--kernel NAME_SUBSTRING] [--all]
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def compile_s(src):
    pkg = [d for d in os.listdir(ROOT) if d.endswith("_amd")][0]
    out = os.path.join(tempfile.mkdtemp(), "k.s")
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-x", "hip",
           "-munsafe-fp-atomics", "--offload-device-only", "-S", "-I", os.path.join(ROOT, pkg, "csrc"), src, "-o", out]
    subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    return open(out).read()


def audit(asm, kfilter=None, show_all=False):
    for m in re.finditer(r"^(_Z\w+):", asm, re.M):
        name = m.group(1)
        if kfilter and kfilter not in name:
            continue
        i = m.end()
        j = asm.find(".Lfunc_end", i)
        body = asm[i:j].splitlines()
        # block membership from hipcc's loop annotations: a block label line carries
        # "Loop Header: Depth=d" (header BBx_y itself) or "in Loop: Header=BBx_y" / "Parent Loop BBx_y"
        loops = {}
        cur = set()
        for l in body:
            lab = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):", l)
            if lab or l.startswith("; =>"):
                if lab:
                    cur = set()
                    if "Loop Header" in l:
                        cur.add(lab.group(1).lstrip("."))
                for hm in re.finditer(r"(?:Header=|Parent Loop )(BB\d+_\d+)", l):
                    cur.add("L" + hm.group(1))
                for k in cur:
                    loops.setdefault(k, {"lines": 0, "inasm": False, "waits": [], "vmem": 0})
            for k in cur:
                d = loops[k]
                d["lines"] += 1
                if "ASMSTART" in l:
                    d["inasm"] = True
                if "ASMEND" in l:
                    d["inasm"] = False
                if re.search(r"buffer_load|global_load|buffer_store|global_store", l):
                    d["vmem"] += 1
                if "s_waitcnt" in l and "vmcnt" in l and not d["inasm"]:
                    d["waits"].append(re.search(r"vmcnt\(\d+\)", l).group(0))
        for k, d in loops.items():
            if (d["waits"] and d["vmem"]) or show_all:
                short = re.sub(r"EEv.*|EvN.*", "", name)
                print(f"{short[:60]:60s} loop {k:10s} {d['lines']:5d} lines  vmem {d['vmem']:3d}  compiler waits {d['waits']}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--kernel", default=None)
    ap.add_argument("--all", action="store_true")
    a = ap.parse_args()
    audit(compile_s(a.src), a.kernel, a.all)


if __name__ == "__main__":
    sys.exit(main())
