"""Code-generation checks on the hand-scheduled kernels (CPU: hipcc cross-compiles gfx950 assembly).

attention.hip loads Q with inline-asm global_load_dwordx4 so that hipcc does not wait vmcnt(0) (draining
the K/V LDS-DMA of tiles 1-2) before Q's first use; the wait is the counted `s_waitcnt vmcnt(4*CPW)`
after tiles 1-2 are issued. hipcc's waitcnt pass cannot see those loads, so correctness rests on no
instruction touching the Q registers between the loads and that wait (a copy, a move or a spill would
read them before they land). This test pins that in the emitted code of every attn16_kernel instance.
"""

import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "f5-tts_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-munsafe-fp-atomics", "-ffp-contract=fast-honor-pragmas",
         "-mllvm", "-disable-promote-alloca-to-lds=1", "--cuda-device-only", "-S"]


def _asm(src, tmp_path):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    out = tmp_path / (os.path.basename(src) + ".s")
    subprocess.run([HIPCC, *FLAGS, os.path.join(CSRC, src), "-o", str(out)], check=True, capture_output=True,
                   timeout=300)
    return out.read_text().splitlines()


def _regs(text):
    """VGPR numbers named in an operand string (vN and v[a:b])."""
    regs = set()
    for a, b in re.findall(r"\bv\[(\d+):(\d+)\]", text):
        regs.update(range(int(a), int(b) + 1))
    for a in re.findall(r"\bv(\d+)\b", text):
        regs.add(int(a))
    return regs


def _functions(lines):
    cur, out = None, {}
    for ln in lines:
        m = re.match(r"^(_Z\S*attn16_kernel\S*):(\s|$)", ln)
        if m:
            cur = m.group(1)
            out[cur] = []
            continue
        if cur and (ln.startswith("\t.size\t" + cur) or ln.startswith(".Lfunc_end")):
            cur = None
        elif cur:
            out[cur].append(ln.strip())
    return out


def test_attention_q_registers_untouched_until_counted_wait(tmp_path):
    funcs = _functions(_asm("attention.hip", tmp_path))
    assert len(funcs) >= 2, list(funcs)  # bf16 and fp16 (prescaled and not)
    for name, body in funcs.items():
        loads = [i for i, ln in enumerate(body)
                 if re.match(r"global_load_dwordx4 v\[\d+:\d+\], v\[\d+:\d+\], off( offset:(32|64|96))?$", ln)]
        assert len(loads) == 4, (name, [body[i] for i in loads])
        qregs = set()
        for i in loads:
            qregs |= _regs(body[i].split(",")[0])
        assert len(qregs) == 16, (name, qregs)
        wait = next(i for i in range(loads[-1] + 1, len(body)) if body[i].startswith("s_waitcnt vmcnt("))
        assert body[wait] == "s_waitcnt vmcnt(4)", (name, body[wait])  # 4 * CPW, CPW = 1 with 8 waves
        for i in range(loads[0] + 1, wait):
            if i in loads or body[i].startswith(";"):
                continue
            assert not (_regs(body[i]) & qregs), (name, body[i])


def test_attention_asm_builds_without_scratch(tmp_path):
    """No attn16_kernel instance spills to scratch (a spill would also break the hand-counted waits)."""
    sizes = {}
    for ln in _asm("attention.hip", tmp_path):
        m = re.match(r"\s*\.set\s+(_Z\S*attn16_kernel\S*)\.private_seg_size,\s*(\d+)", ln)
        if m:
            sizes[m.group(1)] = int(m.group(2))
    assert len(sizes) >= 2 and all(v == 0 for v in sizes.values()), sizes


def test_fp16_gemm_epilogues_round_through_fp32(tmp_path):
    """No fp16 GEMM instance folds an epilogue product into its fp16 conversion (v_fma_mix rounds the
    product once, straight to fp16; the packed fast epilogues round it to fp32 first), so every tile
    configuration stores the same bits (test_sample_bitwise_identical_across_tile_configs[fp16])."""
    lines = _asm("gemm_f16_a.hip", tmp_path)
    cur, kernels, mixed = None, 0, set()
    for ln in lines:
        m = re.match(r"^(_Z\S*gemm\S*_kernel\S*):(\s|$)", ln)
        if m:
            cur = m.group(1)
            kernels += 1
        elif cur and "v_fma_mix" in ln:
            mixed.add(cur)
    assert kernels >= 10 and not mixed, (kernels, sorted(mixed))


@pytest.mark.parametrize("src", ["attention.hip", "gemm_bf16_a.hip"])
def test_lds_dma_never_in_a_waterfall_loop(src, tmp_path):
    """Every LDS-DMA piece (`buffer_load_dwordx4 ... lds`) takes its buffer descriptor from scalar registers the
    compiler can prove wave-uniform. A descriptor it cannot (e.g. an extent computed on the VALU) makes hipcc wrap
    each piece in a waterfall loop: v_readfirstlane x4, a compare, s_and_saveexec, the load, s_xor exec, branch
    back (cdna_hip_programming.md T20; round 5's per-tile attention descriptors did this until the extent went
    through readfirstlane)."""
    lines = [ln.strip() for ln in _asm(src, tmp_path)]
    dma = [i for i, ln in enumerate(lines) if ln.startswith("buffer_load_dwordx4") and ln.endswith(" lds")]
    assert len(dma) > 10, len(dma)
    bad = []
    for i in dma:
        window = lines[max(0, i - 8):i]
        if any(w.startswith("s_and_saveexec") for w in window) or \
                sum(w.startswith("v_readfirstlane_b32") for w in window) >= 4:
            bad.append((i, lines[i]))
    assert not bad, bad[:5]
