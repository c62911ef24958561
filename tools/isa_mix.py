"""Static instruction mix of a kernel's simulation loop, phase by phase (diagnostic, CPU only).

Compiles one libmzh source to gfx950 assembly with the library's own flags (build.FLAGS plus its
build.SOURCE_FLAGS entry), finds the kernel, takes the innermost loop that holds at least MIN_BARRIERS
workgroup barriers (the cooperative kernel's simulation loop) -- or, with --loop-mfma, the smallest loop
holding at least that many MFMAs -- and prints the MFMA / VALU / SALU / LDS / VMEM counts between its
barriers plus the loop's most frequent VALU opcodes.  Static counts: a phase's code for every wave's
branch, not executed instructions; DESIGN.md §8 (round 5) compares builds with it.

  python tools/isa_mix.py                                  # mzh_search.hip, the 8,192-root instantiation
  python tools/isa_mix.py --kernel _Z17mzh_search_kernelILi16ELb0ELb1ELb1ELb0EEv6MzhNet15MzhSearchParams
  python tools/isa_mix.py --extra=-mllvm,-amdgpu-use-amdgpu-trackers=1    # an A/B flag on top
"""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from muzero_hanoi_amd import build  # noqa: E402

DEFAULT_KERNEL = "_Z17mzh_search_kernelILi32ELb0ELb1ELb1ELb0EEv6MzhNet15MzhSearchParams"


def compile_asm(src, extra):
    out = os.path.join(tempfile.mkdtemp(prefix="mzh_isa_"), os.path.basename(src) + ".s")
    flags = [f for f in build.FLAGS if f not in ("-fPIC",)] + build.SOURCE_FLAGS.get(os.path.basename(src), []) + extra
    cmd = [build.HIPCC, *flags, "--cuda-device-only", "-S", os.path.join(build.CSRC, src), "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise SystemExit(r.stderr)
    return open(out).read().split("\n")


def kind(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    return "vmem"


def instrs(lines):
    for s in lines:
        s = s.strip()
        if s and not s.startswith((";", ".")) and not s.endswith(":"):
            yield s.split()[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default="mzh_search.hip")
    ap.add_argument("--kernel", default=DEFAULT_KERNEL)
    ap.add_argument("--min-barriers", type=int, default=5)
    ap.add_argument("--extra", default="", help="comma-separated extra compiler flags")
    a = ap.parse_args()
    T = compile_asm(a.src, [f for f in a.extra.split(",") if f])
    st = next(i for i, l in enumerate(T) if l.startswith(a.kernel + ":"))
    en = next(i for i, l in enumerate(T) if i > st and re.match(r"^_Z\w+:", l))
    L = T[st:en]
    labels = {m.group(1): i for i, l in enumerate(L) for m in [re.match(r"^(\.LBB\w+):", l)] if m}
    best = None
    for i, l in enumerate(L):
        m = re.match(r"\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\w+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            b0 = labels[m.group(1)]
            nb = sum(1 for s in L[b0:i + 1] if s.strip() == "s_barrier")
            if nb >= a.min_barriers and (best is None or i - b0 < best[1] - best[0]):
                best = (b0, i)
    if best is None:
        raise SystemExit("no loop with that many barriers")
    b0, b1 = best
    bars = [i for i in range(b0, b1 + 1) if L[i].strip() == "s_barrier"]
    total = collections.Counter()
    prev = b0
    print(f"{a.kernel}: simulation loop, lines {b0}-{b1}, {len(bars)} barriers")
    for e in bars + [b1]:
        c = collections.Counter(kind(op) for op in instrs(L[prev:e]))
        total += c
        print(f"  phase lines {prev:6d}-{e:6d}: " + ", ".join(f"{k} {c[k]}" for k in ("mfma", "valu", "salu", "lds", "vmem")))
        prev = e
    print("  loop total: " + ", ".join(f"{k} {total[k]}" for k in ("mfma", "valu", "salu", "lds", "vmem")))
    v = collections.Counter(op for op in instrs(L[b0:b1]) if kind(op) == "valu")
    print("  top VALU opcodes: " + ", ".join(f"{op} {n}" for op, n in v.most_common(12)))


if __name__ == "__main__":
    main()
