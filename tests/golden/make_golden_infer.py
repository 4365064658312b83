"""Golden vectors for the host orchestration of inference (tests/test_infer.py), produced by the
REFERENCE's own `chunk_text` and `infer_batch_process` (src/f5_tts/infer/utils_infer.py:73-103,
440-596) with deterministic fake model/vocoder (tests/infer_fakes.py).

Run in the build container only (needs /root/reference, read-only):
    python tests/golden/make_golden_infer.py
Absent third-party modules get stubs; `rjieba.cut` is given this build's `segment_words`
(the segmenter itself stays parity-unpinned), torchaudio's Resample is not exercised (24 kHz
inputs). Only outputs are stored.
"""

from __future__ import annotations

import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "f5-tts_amd"), os.path.join(REPO, "tests")]
sys.dont_write_bytecode = True

from f5_tts_amd.infer import segment_words  # noqa: E402
from infer_fakes import FakeModel, FakeVocoder, ref_audios  # noqa: E402

CHUNK_CASES = [
    ("Hello world. This is a test, with commas; and colons: ok! Done?", 20),
    ("Short.", 135),
    ("A very long sentence without any punctuation that keeps going and going beyond the limit", 30),
    ("你好，世界。这是一个测试！English mixed in. 再见？", 24),
    ("First.Second.  Third!   Fourth", 10),
    ("", 50),
    ("One, two, three, four, five, six, seven, eight, nine, ten.", 12),
]

INFER_CASES = [
    # ref_text, gen batches, speed, fix_duration, target_rms scale of the ref wave, cross-fade
    ("Some call me nature, others call me mother nature.",
     ["I don't really care what you call me.", "I've been a silent spectator, watching species evolve.",
      "Hi."], 1.0, None, 0.05, 0.15),
    ("Reference text", ["Generated; with “quotes” and ‘marks’."], 0.8, None, 0.3, 0.15),
    ("ref", ["abc def ghi", "jkl mno pqr stu"], 1.0, 3.0, 0.02, 0.0),
    ("ref text.", ["tiny", "x" * 40], 1.2, None, 0.2, 5.0),
]


STRIDE = 7


def install_shims():
    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    mod("torchaudio", transforms=types.SimpleNamespace(), load=None)
    lib = mod("librosa")
    lib.filters = mod("librosa.filters", mel=lambda **k: None)
    mod("rjieba", cut=segment_words)
    mod("pypinyin", Style=types.SimpleNamespace(TONE3=3), lazy_pinyin=lambda s, **k: [f"py{ord(c)}" for c in s])
    pd = mod("pydub", AudioSegment=object)
    pd.silence = mod("pydub.silence")
    mod("vocos", Vocos=object)
    mod("soundfile")
    mod("transformers", pipeline=None)  # ASR (whisper) pipeline: off this path
    mod("f5_tts.model.trainer", Trainer=object)
    xt = mod("x_transformers", RMSNorm=object)  # backbones are imported but not used here
    xt.x_transformers = mod("x_transformers.x_transformers", RotaryEmbedding=object, apply_rotary_pos_emb=None)
    mod("torchdiffeq", odeint=None)
    sys.path.insert(0, "/root/reference/src")


def main():
    install_shims()
    from f5_tts.infer import utils_infer as ui

    out = {"chunk": [[t, m, ui.chunk_text(t, max_chars=m)] for t, m in CHUNK_CASES]}
    from f5_tts.model.utils import convert_char_to_pinyin

    pin_cases = ["Hello, world!", "it's a “test”; ok", "mixed 中文 text", "a:b  c\"d", "数字123和abc"]
    out["pinyin"] = [[t, convert_char_to_pinyin([t])[0]] for t in pin_cases]
    arrays = {}
    out["infer"] = []
    audios = ref_audios([c[4] for c in INFER_CASES])
    for i, (ref_text, batches, speed, fix_dur, amp, xfade) in enumerate(INFER_CASES):
        audio = audios[i]
        model, voc = FakeModel(), FakeVocoder()
        gen = ui.infer_batch_process((audio, 24000), ref_text, batches, model, voc, progress=None, nfe_step=16,
                                     cfg_strength=2.0, sway_sampling_coef=-1.0, speed=speed, fix_duration=fix_dur,
                                     cross_fade_duration=xfade, device="cpu")
        wav, sr, spec = next(gen)
        arrays[f"wav{i}"] = np.asarray(wav, np.float32)[::STRIDE]  # every STRIDE-th sample (size)
        out["infer"].append({"sr": sr, "calls": sorted(model.calls), "wav_len": len(wav),
                             "wav_sum": float(np.sum(np.asarray(wav, np.float64)))})
        arrays[f"spec{i}"] = np.asarray(spec, np.float32)
        # streaming form (socket server path)
        model2 = FakeModel()
        chunks = list(ui.infer_batch_process((audio, 24000), ref_text, batches, model2, voc, progress=None,
                                             nfe_step=16, speed=speed, fix_duration=fix_dur, device="cpu",
                                             streaming=True, chunk_size=3000))
        arrays[f"stream{i}"] = np.concatenate([c for c, _ in chunks]).astype(np.float32)[::STRIDE]
        out["infer"][-1]["stream_lens"] = [len(c) for c, _ in chunks]
    np.savez_compressed(os.path.join(HERE, "infer_host.npz"), **arrays)
    with open(os.path.join(HERE, "infer_host.json"), "w") as f:
        json.dump(out, f, indent=1, ensure_ascii=False)
    print("wrote infer_host.npz / infer_host.json")


if __name__ == "__main__":
    main()
