"""Checkpoint formats: reference-layout EMA / raw checkpoints, as .safetensors and
as torch .pt, load into the engine-backed CFM with the reference's key rules (utils_infer.py:188-232).
CPU only (loading is host work; the engine is built from these parameters on first use)."""

import pytest
import torch

import golden_cases as gc
from f5_tts_amd import checkpoint, synthetic
from f5_tts_amd.model import CFM, DiT


def _model():
    arch = gc.arch_of("tiny")
    kw = {k: v for k, v in arch.items() if k not in ("backbone", "text_num_embeds", "mel_dim")}
    return CFM(transformer=DiT(**kw, text_num_embeds=arch["text_num_embeds"], mel_dim=arch["mel_dim"]),
               num_channels=100), arch


def _ref_weights(arch, model):
    W = synthetic.make_weights_torch(arch)
    # reference checkpoints carry x_transformers' persistent rotary buffer
    W["rotary_embed.inv_freq"] = model.transformer.state_dict()["rotary_embed.inv_freq"].clone()
    return W


def _ref_ema_state(arch, model):
    W = _ref_weights(arch, model)
    sd = {f"ema_model.transformer.{k}": v for k, v in W.items()}
    sd["initted"] = torch.tensor(True)
    sd["step"] = torch.tensor(1200)
    sd["ema_model.mel_spec.mel_stft.spectrogram.window"] = torch.ones(1024)  # legacy key (305e3ea patch)
    return sd, W


@pytest.mark.parametrize("fmt", ["safetensors", "pt"])
def test_ema_checkpoint_loads_with_reference_rules(tmp_path, fmt):
    model, arch = _model()
    sd, W = _ref_ema_state(arch, model)
    path = tmp_path / f"model_1200.{fmt}"
    if fmt == "safetensors":
        from safetensors.torch import save_file

        save_file({k: v.contiguous() for k, v in sd.items()}, str(path))
    else:
        torch.save({"ema_model_state_dict": sd, "model_state_dict": {}}, str(path))
    m = checkpoint.load_checkpoint(model, str(path), device="cpu", dtype=torch.float32)
    got = m.transformer.state_dict()
    for k, v in W.items():
        assert torch.equal(got[k], v.float()), k


def test_raw_checkpoint_and_default_dtype(tmp_path):
    model, arch = _model()
    W = _ref_weights(arch, model)
    path = tmp_path / "raw.pt"
    torch.save({"model_state_dict": {f"transformer.{k}": v for k, v in W.items()}}, str(path))
    m = checkpoint.load_checkpoint(model, str(path), device="cpu", use_ema=False)
    assert next(m.parameters()).dtype == torch.float32  # CPU device -> fp32 (utils_infer.py:189-196)
    assert m.engine_compute() == "fp32"
    m16 = m.to(torch.float16)
    assert m16.engine_compute() == "fp16"  # the reference's fp16 GPU rule selects the fp16 MFMA mode
    assert m.to(torch.bfloat16).engine_compute() == "bf16"


def test_missing_key_is_an_error(tmp_path):
    model, arch = _model()
    sd, W = _ref_ema_state(arch, model)
    sd.pop(next(k for k in sd if k.startswith("ema_model.transformer.")))
    path = tmp_path / "broken.pt"
    torch.save({"ema_model_state_dict": sd}, str(path))
    with pytest.raises(RuntimeError):
        checkpoint.load_checkpoint(model, str(path), device="cpu", dtype=torch.float32)
