"""Per-kernel ISA lint for the lgx HIP sources (container-side, no GPU): compiles each source to
gfx950 assembly and counts, per kernel, the loads wrapped in a lane-divergent branch that wait on
their own result right away (s_and_saveexec ... ds_read / global_load ... s_waitcnt): each is one
exposed memory round trip per execution ("a rule that recurs in every kernel").
Usage: python tools/isa_lint.py [source.hip ...]"""
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "legged_gym_amd", "csrc")
SLP_OFF = {"lgx_physics.hip", "lgx_gemm_split.hip", "lgx_gemm_x3p.hip", "lgx_gemm_tn.hip", "lgx_mlp_x3.hip"}


def kernels(asm):
    for m in re.finditer(r"^(\S+):\s*\n(?:.*\n)*?\.Lfunc_end", asm, re.M):
        pass
    out = {}
    for name in re.findall(r"^\s*\.globl\s+(\S+)", asm, re.M):
        start = asm.find("\n" + name + ":")
        if start < 0:
            continue
        end = asm.find(".Lfunc_end", start)
        out[name] = [l.strip() for l in asm[start:end].splitlines()
                     if l.strip() and not l.strip().startswith((".", ";"))]
    return out


def wrapped_loads(ins):
    n = 0
    for i, l in enumerate(ins):
        if l.startswith("s_and_saveexec"):
            w = ins[i + 1:i + 5]
            if any(x.startswith(("ds_read", "global_load", "buffer_load")) for x in w) and \
               any(x.startswith("s_waitcnt") for x in w):
                n += 1
    return n


def main(paths):
    paths = paths or sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    with tempfile.TemporaryDirectory() as td:
        for p in paths:
            out = os.path.join(td, os.path.basename(p) + ".s")
            flags = ["-fno-slp-vectorize"] if os.path.basename(p) in SLP_OFF else []
            subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-munsafe-fp-atomics",
                            "--cuda-device-only", "-S", *flags, p, "-o", out], check=True, capture_output=True)
            for name, ins in kernels(open(out).read()).items():
                w = wrapped_loads(ins)
                if w:
                    print(f"{os.path.basename(p)}: {name[:70]}: {w} branch-wrapped loads ({len(ins)} instructions)")


if __name__ == "__main__":
    main(sys.argv[1:])
