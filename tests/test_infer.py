"""Inference host surface (f5_tts_amd.infer / .api) — the reference's utils_infer.py / api.py.

CPU tests pin the orchestration (chunking, text conversion, duration rule, RMS handling,
cross-fade, streaming) against the reference's own functions run on deterministic fake
model/vocoder (tests/golden/make_golden_infer.py). The GPU test runs `F5TTS.infer` end to end
on the HIP engine (mel front end, CFM.sample, Vocos) with synthetic weights.
"""

from __future__ import annotations

import json
import os

import numpy as np
import pytest
import torch

from f5_tts_amd import infer
from infer_fakes import FakeModel, FakeVocoder, ref_audios

GOLD = os.path.join(os.path.dirname(__file__), "golden")

INFER_CASES = [
    ("Some call me nature, others call me mother nature.",
     ["I don't really care what you call me.", "I've been a silent spectator, watching species evolve.",
      "Hi."], 1.0, None, 0.05, 0.15),
    ("Reference text", ["Generated; with “quotes” and ‘marks’."], 0.8, None, 0.3, 0.15),
    ("ref", ["abc def ghi", "jkl mno pqr stu"], 1.0, 3.0, 0.02, 0.0),
    ("ref text.", ["tiny", "x" * 40], 1.2, None, 0.2, 5.0),
]
STRIDE = 7


@pytest.fixture(scope="module")
def gold():
    with open(os.path.join(GOLD, "infer_host.json"), encoding="utf-8") as f:
        j = json.load(f)
    return j, np.load(os.path.join(GOLD, "infer_host.npz"))


def test_chunk_text_matches_reference(gold):
    j, _ = gold
    for text, max_chars, want in j["chunk"]:
        assert infer.chunk_text(text, max_chars=max_chars) == want, text


def test_convert_char_to_pinyin_matches_reference(gold):
    j, _ = gold
    fake_py = lambda s: [f"py{ord(c)}" for c in s]  # the golden script's pypinyin stand-in
    for text, want in j["pinyin"]:
        assert infer.convert_char_to_pinyin([text], to_pinyin=fake_py)[0] == want, text


def test_infer_batch_process_matches_reference(gold):
    j, z = gold
    audios = ref_audios([c[4] for c in INFER_CASES])
    for i, (ref_text, batches, speed, fix_dur, _amp, xfade) in enumerate(INFER_CASES):
        model = FakeModel()
        wav, sr, spec = next(infer.infer_batch_process((audios[i], 24000), ref_text, batches, model, FakeVocoder(),
                                                       nfe_step=16, cfg_strength=2.0, sway_sampling_coef=-1.0,
                                                       speed=speed, fix_duration=fix_dur, cross_fade_duration=xfade,
                                                       device="cpu"))
        g = j["infer"][i]
        assert sr == g["sr"]
        assert sorted(list(c) for c in model.calls) == [list(c) for c in g["calls"]]
        assert len(wav) == g["wav_len"]
        np.testing.assert_allclose(np.asarray(wav, np.float32)[::STRIDE], z[f"wav{i}"], rtol=1e-5, atol=1e-6)
        assert abs(float(np.sum(np.asarray(wav, np.float64))) - g["wav_sum"]) <= 1e-6 * max(1.0, abs(g["wav_sum"]))
        np.testing.assert_allclose(spec, z[f"spec{i}"], rtol=1e-6, atol=1e-6)
        chunks = list(infer.infer_batch_process((audios[i], 24000), ref_text, batches, FakeModel(), FakeVocoder(),
                                                nfe_step=16, speed=speed, fix_duration=fix_dur, device="cpu",
                                                streaming=True, chunk_size=3000))
        assert [len(c) for c, _ in chunks] == g["stream_lens"]
        np.testing.assert_allclose(np.concatenate([c for c, _ in chunks])[::STRIDE], z[f"stream{i}"],
                                   rtol=1e-5, atol=1e-6)


def test_infer_process_chunks_by_reference_rate():
    """utils_infer.py:402-404: max_chars = ref bytes / ref seconds * (22 - ref seconds) * speed."""
    audio = ref_audios([0.1])[0]  # 1 s at 24 kHz
    model = FakeModel()
    text = "Alpha beta gamma. " * 30
    wav, sr, spec = infer.infer_process((audio, 24000), "Ten bytes.", text, model, FakeVocoder(),
                                        show_info=lambda *a: None, nfe_step=4)
    want = infer.chunk_text(text, max_chars=int(10 / 1.0 * 21 * 1.0))
    assert len(model.calls) == len(want) > 1
    assert sorted(c[0] for c in model.calls) == sorted("Ten bytes. " + w for w in want)
    assert spec.shape[0] == 100 and sr == 24000 and wav.ndim == 1
    none = infer.infer_process((audio, 24000), "Ten bytes.", "", model, FakeVocoder(), show_info=lambda *a: None)
    assert none == (None, 24000, None)


def test_cross_fade_edges():
    a, b = np.ones(10), np.zeros(4)
    np.testing.assert_array_equal(infer.cross_fade([a, b], 0.0), np.concatenate([a, b]))
    out = infer.cross_fade([a, b], 1.0, sample_rate=100)  # overlap clipped to the shorter wave (4)
    assert len(out) == 10
    np.testing.assert_allclose(out[-4:], np.linspace(1, 0, 4))
    assert len(infer.cross_fade([a, np.zeros(0)], 1.0, sample_rate=100)) == 10


def test_resample_properties():
    sr0, sr1 = 16000, 24000
    t = torch.arange(sr0) / sr0
    x = torch.sin(2 * torch.pi * 440 * t)[None]
    y = infer.resample(x, sr0, sr1)
    assert y.shape == (1, 24000)
    # a 440 Hz tone keeps its amplitude and frequency (interior, away from the padded edges)
    ty = torch.arange(24000) / sr1
    ref = torch.sin(2 * torch.pi * 440 * ty)[None]
    assert (y[:, 200:-200] - ref[:, 200:-200]).abs().max() < 2e-3
    # constant signal stays constant; identity when rates match; ceil length rule
    assert (infer.resample(torch.ones(2, 3000), 44100, 24000)[:, 100:-100] - 1).abs().max() < 2e-3
    assert infer.resample(x, 24000, 24000) is x
    assert infer.resample(torch.zeros(1, 1001), 44100, 24000).shape[-1] == int(np.ceil(1001 * 24000 / 44100))


def test_wav_round_trip(tmp_path):
    w = (np.sin(np.arange(5000) * 0.01) * 0.5).astype(np.float32)
    p = str(tmp_path / "a.wav")
    infer.save_wav(p, w, 22050)
    a, sr = infer.load_audio(p)
    assert sr == 22050 and a.shape == (1, 5000)
    assert np.abs(a[0].numpy() - w).max() < 1.0 / 32767 + 1e-6


def test_reference_example_wav_loads():
    p = "/root/reference/src/f5_tts/infer/examples/basic/basic_ref_en.wav"
    if not os.path.exists(p):
        pytest.skip("reference tree absent")
    a, sr = infer.load_audio(p)
    assert a.ndim == 2 and sr > 0 and a.shape[-1] > sr and float(a.abs().max()) <= 1.0


def test_api_requires_local_assets():
    from f5_tts_amd.api import F5TTS

    with pytest.raises(ValueError):
        F5TTS(model="DiT_tiny", ckpt_file="synthetic", vocoder_local_path=None)
    with pytest.raises(KeyError):
        F5TTS(model="nope", ckpt_file="synthetic", vocoder_local_path="synthetic")


@pytest.mark.gpu
def test_api_infer_end_to_end_gpu(tmp_path):
    """F5TTS.infer on the HIP engine: mel front end, CFM.sample, Vocos decode, cross-fade, WAV export.
    Deterministic for a fixed seed; the wave length follows the duration rule per chunk."""
    from f5_tts_amd.api import F5TTS

    tts = F5TTS(model="DiT_tiny", ckpt_file="synthetic", vocoder_local_path="synthetic", device="cuda")
    ref = ref_audios([0.1])[0]
    kw = dict(show_info=lambda *a: None, nfe_step=4, cross_fade_duration=0.0)
    gen = "Hello there. General Kenobi!"
    wav, sr, spec = tts.infer((ref, 24000), "Reference words.", gen, seed=3, file_wave=str(tmp_path / "o.wav"), **kw)
    wav2, _, _ = tts.infer((ref, 24000), "Reference words.", gen, seed=3, **kw)
    assert sr == 24000 and np.isfinite(wav).all() and np.array_equal(wav, wav2)
    ref_frames = ref.shape[-1] // 256
    ref_text = "Reference words. "
    chunks = infer.chunk_text(gen, max_chars=int(len(ref_text.strip()) / 1.0 * 21))
    frames = [int(ref_frames / len(ref_text) * len(c)) for c in chunks]
    assert spec.shape == (100, sum(frames))
    assert len(wav) == sum((f - 1) * 256 for f in frames)
    a, sr2 = infer.load_audio(str(tmp_path / "o.wav"))
    assert sr2 == 24000 and a.shape[-1] == len(wav)
