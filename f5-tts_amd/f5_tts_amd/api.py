"""`F5TTS` — the reference's one-object API (src/f5_tts/api.py:23-150) on the HIP engine.

Same constructor and `infer()` arguments and return value `(wave, sr, spectrogram)`. No network
in this environment, so `ckpt_file`, `vocab_file` and `vocoder_local_path` must point at local
files (the reference downloads them when empty); `ckpt_file="synthetic"` builds hash-PRNG
weights of the named architecture and `vocoder_local_path="synthetic"` a synthetic Vocos, which
is what the benchmarks and tests use. `transcribe()` (whisper ASR) is out of scope.
"""

from __future__ import annotations

import random
import sys

import torch

from . import configs, infer
from .checkpoint import load_model
from .model import CFM, DiT, UNetT

_BACKBONES = {"DiT": DiT, "UNetT": UNetT}


def seed_everything(seed: int = 0) -> None:
    """model/utils.py:19-29 (python, torch CPU and device generators)."""
    random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


def _synthetic_model(model: str, device: str, vocab_size: int = configs.VOCAB_SIZE):
    from . import synthetic

    arch = configs.get_arch(model, text_num_embeds=vocab_size)
    kw = {k: v for k, v in arch.items() if k not in ("backbone", "text_num_embeds", "mel_dim")}
    net = _BACKBONES[arch["backbone"]](**kw, text_num_embeds=arch["text_num_embeds"], mel_dim=arch["mel_dim"])
    net.load_state_dict(synthetic.make_weights_torch(arch), strict=False)
    # printable ASCII at 0..94 (space first, as the reference vocab.txt starts with " "), fillers after
    vocab = {chr(32 + i) if i < 95 else f"<{i}>": i for i in range(vocab_size)}
    m = CFM(transformer=net, num_channels=arch["mel_dim"], vocab_char_map=vocab)
    dtype = torch.float16 if device.startswith("cuda") else torch.float32
    return m.to(dtype).to(device)


class F5TTS:
    def __init__(self, model: str = "F5TTS_v1_Base", ckpt_file: str = "", vocab_file: str = "",
                 ode_method: str = "euler", use_ema: bool = True, vocoder_local_path: str | None = None,
                 device: str | None = None, hf_cache_dir=None):
        if model not in configs.PRESETS:
            raise KeyError(f"unknown model {model!r}; known: {sorted(configs.PRESETS)}")
        self.mel_spec_type = "vocos"
        self.target_sample_rate = infer.target_sample_rate
        self.ode_method = ode_method
        self.use_ema = use_ema
        self.device = device or ("cuda" if torch.cuda.is_available() else "cpu")
        if vocoder_local_path is None:
            raise ValueError("no network here: vocoder_local_path must name a local vocos-mel-24khz directory "
                             "(or 'synthetic')")
        self.vocoder = infer.load_vocoder(self.mel_spec_type, True, vocoder_local_path, self.device, hf_cache_dir)
        if ckpt_file == "synthetic":
            self.ema_model = _synthetic_model(model, self.device)
        elif ckpt_file:
            arch = configs.get_arch(model)
            cfg = {k: v for k, v in arch.items() if k not in ("backbone", "text_num_embeds", "mel_dim")}
            self.ema_model = load_model(_BACKBONES[arch["backbone"]], cfg, ckpt_file, self.mel_spec_type, vocab_file,
                                        ode_method, use_ema, self.device)
        else:
            raise ValueError("no network here: ckpt_file must name a local checkpoint (or 'synthetic')")

    def transcribe(self, ref_audio, language=None):
        raise NotImplementedError("ASR transcription (whisper) is outside the sampling engine; pass ref_text")

    def export_wav(self, wav, file_wave, remove_silence=False):
        if remove_silence:
            raise NotImplementedError("silence removal needs pydub (absent)")
        infer.save_wav(file_wave, wav, self.target_sample_rate)

    def infer(self, ref_file, ref_text, gen_text, show_info=print, progress=None, target_rms=0.1,
              cross_fade_duration=0.15, sway_sampling_coef=-1, cfg_strength=2, nfe_step=32, speed=1.0,
              fix_duration=None, remove_silence=False, file_wave=None, file_spec=None, seed=None):
        """api.py:98-150: seed, synthesize (chunked, cross-faded), optionally write the wave."""
        if seed is None:
            seed = random.randint(0, sys.maxsize)
        seed_everything(seed)
        self.seed = seed
        if not ref_text or not ref_text.strip():
            raise ValueError("ref_text is required (ASR transcription is out of scope)")
        wav, sr, spec = infer.infer_process(ref_file, ref_text, gen_text, self.ema_model, self.vocoder,
                                            self.mel_spec_type, show_info=show_info, progress=progress,
                                            target_rms=target_rms, cross_fade_duration=cross_fade_duration,
                                            nfe_step=nfe_step, cfg_strength=cfg_strength,
                                            sway_sampling_coef=sway_sampling_coef, speed=speed,
                                            fix_duration=fix_duration, device=self.device)
        if file_wave is not None:
            self.export_wav(wav, file_wave, remove_silence)
        if file_spec is not None:
            raise NotImplementedError("spectrogram PNG export (matplotlib) is not part of the engine")
        return wav, sr, spec
