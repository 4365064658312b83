"""The C-ABI boundary: libf5h.so loads, exports exactly what include/f5h.h declares, and the
ctypes mirrors have the C layout (no GPU needed, no compute calls)."""

import ctypes
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "f5h.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(f5h_[a-z_]+)\s*\(", src)))


def test_header_declares_the_python_export_list():
    from f5_tts_amd import _lib

    assert sorted(_lib.EXPORTS) == _declared()


def test_library_loads_and_exports_every_symbol():
    from f5_tts_amd import _lib

    L = _lib.lib()
    for name in _declared():
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (f5h_\w+)", out))
    assert set(_declared()) <= exported
    assert L.f5h_version().decode().startswith("f5h")


def test_library_is_gfx950_code():
    from f5_tts_amd import _lib

    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in blob


def test_struct_layout_matches_c(tmp_path):
    from f5_tts_amd import _lib

    prog = tmp_path / "layout.c"
    prog.write_text(f"""
#include <stdio.h>
#include <stddef.h>
#include "{HEADER}"
int main(void) {{
  printf("%zu %zu %zu %zu\\n", sizeof(f5h_arch), sizeof(f5h_weight), sizeof(f5h_sample_args), sizeof(f5h_forward_args));
  printf("%zu %zu %zu %zu\\n", offsetof(f5h_sample_args, cfg_strength), offsetof(f5h_sample_args, out),
         offsetof(f5h_forward_args, t), offsetof(f5h_forward_args, pred));
  printf("%zu %zu\\n", sizeof(f5h_vocos_arch), offsetof(f5h_vocos_arch, compute));
  printf("%zu %zu %zu %zu\\n", sizeof(f5h_tensor_view), offsetof(f5h_tensor_view, dtype),
         offsetof(f5h_tensor_view, on_device), offsetof(f5h_tensor_view, numel));
  return 0;
}}""")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", str(prog), "-o", str(exe)], check=True)
    got = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()
    want = [ctypes.sizeof(_lib.Arch), ctypes.sizeof(_lib.Weight), ctypes.sizeof(_lib.SampleArgs),
            ctypes.sizeof(_lib.ForwardArgs), _lib.SampleArgs.cfg_strength.offset, _lib.SampleArgs.out.offset,
            _lib.ForwardArgs.t.offset, _lib.ForwardArgs.pred.offset,
            ctypes.sizeof(_lib.VocosArch), _lib.VocosArch.compute.offset,
            ctypes.sizeof(_lib.TensorView), _lib.TensorView.dtype.offset, _lib.TensorView.on_device.offset,
            _lib.TensorView.numel.offset]
    assert [int(x) for x in got] == want


def test_errors_are_reported_not_crashing():
    """A bad arch is rejected with a message (no device touched before validation)."""
    from f5_tts_amd import _lib

    L = _lib.lib()
    a = _lib.Arch(backbone=0, dim=1000, depth=1, heads=16, dim_head=64, ff_dim=2048, text_dim=512,
                  text_num_embeds=10, mel_dim=100, conv_layers=0, text_mask_padding=1, pe_attn_head=0,
                  attn_mask_enabled=0, compute=1)
    h = ctypes.c_void_p()
    rc = L.f5h_engine_create(ctypes.byref(a), None, 0, 0, ctypes.byref(h))
    assert rc == -1 and b"multiple of 128" in L.f5h_last_error()
    # typed views: a bad dtype or placement flag is rejected before any device work
    good = _lib.Arch(backbone=0, dim=256, depth=1, heads=4, dim_head=64, ff_dim=512, text_dim=128,
                     text_num_embeds=10, mel_dim=100, conv_layers=0, text_mask_padding=1, pe_attn_head=0,
                     attn_mask_enabled=0, compute=1)
    buf = (ctypes.c_float * 4)()
    v = (_lib.TensorView * 1)()
    v[0].name, v[0].data, v[0].dtype, v[0].on_device, v[0].numel = b"w", ctypes.addressof(buf), 7, 0, 4
    rc = L.f5h_engine_create_views(ctypes.byref(good), v, 1, 0, ctypes.byref(h))
    assert rc == -1 and b"dtype" in L.f5h_last_error()
    v[0].dtype, v[0].on_device = _lib.F5H_DT_BF16, 3
    rc = L.f5h_engine_create_views(ctypes.byref(good), v, 1, 0, ctypes.byref(h))
    assert rc == -1 and b"on_device" in L.f5h_last_error()
    va = _lib.VocosArch(100, 500, 1536, 8, 1024, 256, 0)
    rc = L.f5h_vocos_create(ctypes.byref(va), None, 0, 0, ctypes.byref(h))
    assert rc == -1 and b"bad vocos arch" in L.f5h_last_error()


def test_no_cpu_fallback_in_product_path():
    """The product package never imports the oracle."""
    pkg = os.path.join(REPO, "f5-tts_amd", "f5_tts_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                txt = open(os.path.join(root, f)).read()
                assert not re.search(r"^\s*(import|from)\s+oracle", txt, flags=re.M), f
