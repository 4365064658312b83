"""CPU check of the one-wave-per-SIMD attention kernel's register contract: hipcc neither touches
the accumulator registers the kernel owns through inline asm nor spills (tools/audit_attn_asm.py)."""
import os
import shutil
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))


@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="needs hipcc")
def test_attn_pw_kernel_owns_its_accumulator_registers():
    import audit_attn_asm

    n, problems = audit_attn_asm.audit()
    assert n == 4, n  # {bf16, fp16} x {q prescaled, not}
    assert not problems, problems[:5]
