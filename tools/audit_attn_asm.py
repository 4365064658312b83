"""Audit of attn_pw_kernel's register contract (attention.hip): the kernel owns a0..a159 through
inline asm, so hipcc must neither touch an accumulator register itself (a spill or copy there
would silently corrupt O, Q or K) nor spill at all. Compiles attention.hip for gfx950 with
-save-temps into a scratch directory and checks every attn_pw_kernel instantiation.
  python tools/audit_attn_asm.py          (exit 1 on a violation)"""
import glob
import os
import re
import subprocess
import sys
import tempfile

CSRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "f5-tts_amd", "csrc")


def audit():
    problems, kernels = [], 0
    with tempfile.TemporaryDirectory() as tmp:
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-munsafe-fp-atomics",
               "-ffp-contract=fast-honor-pragmas", "-mllvm", "-disable-promote-alloca-to-lds=1", "-mllvm",
               "-amdgpu-mfma-vgpr-form=true", "--save-temps", "-c", os.path.join(CSRC, "attention.hip"),
               "-o", os.path.join(tmp, "a.o")]
        subprocess.run(cmd, check=True, cwd=tmp, capture_output=True)
        asm = open(glob.glob(os.path.join(tmp, "*amdgcn*.s"))[0]).read()
    for m in re.finditer(r"^(_ZN3f5h14attn_pw_kernel\w+):", asm, re.M):
        kernels += 1
        name = m.group(1)
        body = asm[m.end():asm.index(".Lfunc_end", m.end())]
        inside = False
        for line in body.splitlines():
            if ";;#ASMSTART" in line:
                inside = True
            elif ";;#ASMEND" in line:
                inside = False
            elif not inside and (re.search(r"\ba\[?\d", line) or "accvgpr" in line or "scratch_" in line):
                problems.append(f"{name}: compiler code touches the accumulator file or scratch: {line.strip()}")
        meta = asm[asm.index(f".name:           {name}"):]
        spill = int(re.search(r"\.vgpr_spill_count:\s+(\d+)", meta).group(1))
        if spill:
            problems.append(f"{name}: {spill} VGPR spills")
    if kernels == 0:
        problems.append("no attn_pw_kernel instantiation found")
    return kernels, problems


if __name__ == "__main__":
    n, probs = audit()
    print(f"attn_pw_kernel instantiations audited: {n}")
    for p in probs[:20]:
        print(p)
    sys.exit(1 if probs else 0)
