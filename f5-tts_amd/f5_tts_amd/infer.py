"""Host-side inference surface around the HIP sampler: the reference's `infer_process()` family
(src/f5_tts/infer/utils_infer.py) with the same names, arguments, defaults and return values.

What runs where:
* text chunking, character/pinyin conversion, duration rule, RMS normalisation, resampling and
  the cross-fade of the chunk waves are host work (as in the reference);
* the reference wave -> log-mel (`MelSpec`, f5h_mel_*), the whole `CFM.sample` ODE loop
  (f5h_sample) and the Vocos decode (f5h_vocos_decode) run in libf5h.so on the GPU.

Absent third-party pieces and what replaces them:
* `torchaudio.load` -> `load_audio` (PCM/float WAV through the standard-library `wave` reader);
* `torchaudio.transforms.Resample` -> `resample` (restatement of torchaudio's default
  `sinc_interp_hann` kernel, lowpass width 6, rolloff 0.99; parity unpinned: torchaudio is not
  in this image);
* `rjieba.cut` -> `segment_words` (word/whitespace/punctuation split of non-CJK runs, the part of
  jieba's behaviour `convert_char_to_pinyin` depends on; parity unpinned);
* `pypinyin.lazy_pinyin` is used when importable; otherwise Chinese input raises.
* ASR transcription (`transcribe`, whisper through transformers) and pydub silence trimming are
  out of scope: `ref_text` must be given.
"""

from __future__ import annotations

import math
import re
import wave
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

# utils_infer.py:50-65 (inference defaults)
target_sample_rate = 24000
n_mel_channels = 100
hop_length = 256
win_length = 1024
n_fft = 1024
mel_spec_type = "vocos"
target_rms = 0.1
cross_fade_duration = 0.15
ode_method = "euler"
nfe_step = 32
cfg_strength = 2.0
sway_sampling_coef = -1.0
speed = 1.0
fix_duration = None


def _default_device() -> str:
    return "cuda" if torch.cuda.is_available() else "cpu"


# ------------------------------------------------------------------ text front end
def chunk_text(text: str, max_chars: int = 135) -> "list[str]":
    """utils_infer.py:73-103: sentence split after ASCII punctuation + whitespace or after
    full-width punctuation; greedy packing of sentences into chunks of <= max_chars UTF-8 bytes
    (a sentence whose last character is single-byte is followed by a space)."""
    out: "list[str]" = []
    cur = ""
    for sent in re.split(r"(?<=[;:,.!?])\s+|(?<=[；：，。！？])", text):
        if not sent:
            continue
        piece = sent + " " if len(sent[-1].encode("utf-8")) == 1 else sent
        if len(cur.encode("utf-8")) + len(sent.encode("utf-8")) <= max_chars:
            cur += piece
        else:
            if cur:
                out.append(cur.strip())
            cur = piece
    if cur:
        out.append(cur.strip())
    return out


_SEG = re.compile(r"[A-Za-z0-9]+(?:\.\d+)?%?|\s+|.", re.S)
_HAN_RUN = re.compile("([\u3100-\u9fff]+)")


def segment_words(text: str) -> "list[str]":
    """Stand-in for `rjieba.cut` (absent here): CJK runs stay whole (the caller converts them
    character by character), ASCII letters/digits group into words, whitespace runs and every
    other character are their own segments."""
    segs: "list[str]" = []
    for part in _HAN_RUN.split(text):
        if not part:
            continue
        if _HAN_RUN.fullmatch(part):
            segs.append(part)
        else:
            segs.extend(_SEG.findall(part))
    return segs


def _lazy_pinyin(seg: str) -> "list[str]":
    try:
        from pypinyin import Style, lazy_pinyin
    except ImportError as e:  # pragma: no cover - pypinyin is not in this image
        raise NotImplementedError("Chinese text needs pypinyin (absent in this image)") from e
    return lazy_pinyin(seg, style=Style.TONE3, tone_sandhi=True)


def convert_char_to_pinyin(text_list, polyphone: bool = True, segment=segment_words, to_pinyin=_lazy_pinyin):
    """model/utils.py:148-188: per text, translate a few OOV punctuation marks, segment, keep
    pure-ASCII segments as characters (a space before a multi-character segment unless the
    previous token is one of ` :'"`), pinyin (TONE3) for pure CJK segments with a space before
    each Chinese character, character-wise handling of mixed segments."""
    custom_trans = str.maketrans({";": ",", "“": '"', "”": '"', "‘": "'", "’": "'"})

    def is_chinese(c):
        return "\u3100" <= c <= "\u9fff"

    final = []
    for text in text_list:
        chars: "list[str]" = []
        text = text.translate(custom_trans)
        for seg in segment(text):
            nbytes = len(bytes(seg, "UTF-8"))
            if nbytes == len(seg):
                if chars and nbytes > 1 and chars[-1] not in " :'\"":
                    chars.append(" ")
                chars.extend(seg)
            elif polyphone and nbytes == 3 * len(seg):
                py = to_pinyin(seg)
                for i, c in enumerate(seg):
                    if is_chinese(c):
                        chars.append(" ")
                    chars.append(py[i])
            else:
                for c in seg:
                    if ord(c) < 256:
                        chars.extend(c)
                    elif is_chinese(c):
                        chars.append(" ")
                        chars.extend(to_pinyin(c))
                    else:
                        chars.append(c)
        final.append(chars)
    return final


# ------------------------------------------------------------------ audio helpers
def load_audio(path: str) -> "tuple[torch.Tensor, int]":
    """WAV file -> (float32 [channels, samples] in [-1, 1], sample rate), like `torchaudio.load`."""
    with wave.open(path, "rb") as w:
        nch, width, sr, n = w.getnchannels(), w.getsampwidth(), w.getframerate(), w.getnframes()
        raw = w.readframes(n)
    if width == 1:
        a = (np.frombuffer(raw, np.uint8).astype(np.float32) - 128.0) / 128.0
    elif width == 2:
        a = np.frombuffer(raw, "<i2").astype(np.float32) / 32768.0
    elif width == 3:
        b = np.frombuffer(raw, np.uint8).reshape(-1, 3).astype(np.int32)
        v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
        v = np.where(v >= 1 << 23, v - (1 << 24), v)
        a = v.astype(np.float32) / float(1 << 23)
    elif width == 4:
        a = np.frombuffer(raw, "<i4").astype(np.float64) / float(1 << 31)
        a = a.astype(np.float32)
    else:
        raise ValueError(f"unsupported WAV sample width {width}")
    return torch.from_numpy(a.reshape(-1, nch).T.copy()), sr


def save_wav(path: str, wav: np.ndarray, sr: int = target_sample_rate) -> None:
    """float wave in [-1, 1] -> 16-bit PCM WAV (stands in for `soundfile.write`, absent here)."""
    pcm = np.clip(np.asarray(wav, np.float32), -1.0, 1.0)
    pcm = np.round(pcm * 32767.0).astype("<i2")
    with wave.open(path, "wb") as w:
        w.setnchannels(1 if pcm.ndim == 1 else pcm.shape[0])
        w.setsampwidth(2)
        w.setframerate(sr)
        w.writeframes((pcm if pcm.ndim == 1 else pcm.T).tobytes())


def _sinc_resample_kernel(orig: int, new: int, width_taps: int = 6, rolloff: float = 0.99):
    base = min(orig, new) * rolloff
    width = math.ceil(width_taps * orig / base)
    idx = torch.arange(-width, width + orig, dtype=torch.float64)[None, None] / orig
    t = torch.arange(0, -new, -1, dtype=torch.float64)[:, None, None] / new + idx
    t = (t * base).clamp(-width_taps, width_taps)
    window = torch.cos(t * math.pi / width_taps / 2) ** 2
    t = t * math.pi
    k = torch.where(t == 0, torch.ones_like(t), torch.sin(t) / t)
    return (k * window * (base / orig)).float(), width


def resample(wave_t: torch.Tensor, orig_freq: int, new_freq: int) -> torch.Tensor:
    """torchaudio.functional.resample (sinc_interp_hann, lowpass width 6, rolloff 0.99):
    polyphase band-limited interpolation, output length ceil(new * n / orig)."""
    if orig_freq == new_freq:
        return wave_t
    g = math.gcd(int(orig_freq), int(new_freq))
    orig, new = int(orig_freq) // g, int(new_freq) // g
    kernel, width = _sinc_resample_kernel(orig, new)
    shape = wave_t.shape
    x = wave_t.reshape(-1, shape[-1]).float()
    n = x.shape[-1]
    x = torch.nn.functional.pad(x, (width, width + orig))
    y = torch.nn.functional.conv1d(x[:, None], kernel.to(x.device), stride=orig)
    y = y.transpose(1, 2).reshape(x.shape[0], -1)
    y = y[..., : math.ceil(new * n / orig)]
    return y.reshape(*shape[:-1], y.shape[-1])


def cross_fade(waves: "list[np.ndarray]", cross_fade_duration: float = cross_fade_duration,
               sample_rate: int = target_sample_rate) -> np.ndarray:
    """utils_infer.py:552-589: linear fade-out/fade-in over min(duration*sr, both lengths)
    samples between consecutive chunk waves (plain concatenation when that is <= 0)."""
    if cross_fade_duration <= 0:
        return np.concatenate(waves)
    final = waves[0]
    for nxt in waves[1:]:
        n = min(int(cross_fade_duration * sample_rate), len(final), len(nxt))
        if n <= 0:
            final = np.concatenate([final, nxt])
            continue
        mixed = final[-n:] * np.linspace(1, 0, n) + nxt[:n] * np.linspace(0, 1, n)
        final = np.concatenate([final[:-n], mixed, nxt[n:]])
    return final


# ------------------------------------------------------------------ model / vocoder loading
def load_vocoder(vocoder_name: str = "vocos", is_local: bool = False, local_path: str = "", device=None,
                 hf_cache_dir=None):
    """utils_infer.py:106-150 for vocos: `pytorch_model.bin` (weights_only) or
    `model.safetensors` under `local_path` into the HIP Vocos. No network: `is_local` is
    required; `local_path="synthetic"` gives hash-PRNG weights (benchmarks, tests)."""
    from . import vocos as _vocos

    if vocoder_name != "vocos":
        raise NotImplementedError("only the vocos vocoder is on the HIP path (BigVGAN is out of scope)")
    device = device or _default_device()
    voc = _vocos.Vocos(**_vocos.VOCOS_MEL_24KHZ)
    if local_path == "synthetic":
        sd = _vocos.make_weights()
    elif is_local and local_path:
        import os

        st = os.path.join(local_path, "model.safetensors")
        if os.path.exists(st):
            from safetensors.torch import load_file

            sd = load_file(st)
        else:
            sd = torch.load(os.path.join(local_path, "pytorch_model.bin"), map_location="cpu", weights_only=True)
    else:
        raise ValueError("no network here: pass is_local=True with local_path to a vocos-mel-24khz directory")
    voc.load_state_dict(sd)
    return voc.eval().to(device)


# ------------------------------------------------------------------ inference
def infer_process(ref_audio, ref_text, gen_text, model_obj, vocoder, mel_spec_type=mel_spec_type, show_info=print,
                  progress=None, target_rms=target_rms, cross_fade_duration=cross_fade_duration, nfe_step=nfe_step,
                  cfg_strength=cfg_strength, sway_sampling_coef=sway_sampling_coef, speed=speed,
                  fix_duration=fix_duration, device=None):
    """utils_infer.py:384-437: load the reference audio, chunk `gen_text` to what fits a ~22 s
    window at the reference's bytes-per-second, and run `infer_batch_process`.
    `ref_audio` is a WAV path or an `(audio [C, n] tensor, sr)` tuple."""
    audio, sr = load_audio(ref_audio) if isinstance(ref_audio, str) else ref_audio
    secs = audio.shape[-1] / sr
    max_chars = int(len(ref_text.encode("utf-8")) / secs * (22 - secs) * speed)
    batches = chunk_text(gen_text, max_chars=max_chars)
    show_info(f"Generating audio in {len(batches)} batches...")
    if not batches:
        show_info("No text batches to generate.")
        return None, target_sample_rate, None
    return next(infer_batch_process((audio, sr), ref_text, batches, model_obj, vocoder, mel_spec_type=mel_spec_type,
                                    progress=progress, target_rms=target_rms,
                                    cross_fade_duration=cross_fade_duration, nfe_step=nfe_step,
                                    cfg_strength=cfg_strength, sway_sampling_coef=sway_sampling_coef, speed=speed,
                                    fix_duration=fix_duration, device=device))


def infer_batch_process(ref_audio, ref_text, gen_text_batches, model_obj, vocoder, mel_spec_type="vocos",
                        progress=None, target_rms=0.1, cross_fade_duration=0.15, nfe_step=32, cfg_strength=2.0,
                        sway_sampling_coef=-1, speed=1, fix_duration=None, device=None, streaming=False,
                        chunk_size=2048):
    """utils_infer.py:440-596. Generator: yields `(wave, sr, spectrogram)` once (or, with
    `streaming`, `(wave_chunk, sr)` pieces of each batch in order). Per batch: duration
    = ref frames + ref frames / ref bytes * gen bytes / speed (speed 0.3 for < 10-byte text),
    `model_obj.sample` on the raw reference wave, keep the generated frames, Vocos decode,
    undo the RMS boost. Batches run on a thread pool as the reference does (each call is
    re-entrant on the engine)."""
    if mel_spec_type != "vocos":
        raise NotImplementedError("only the vocos mel/vocoder pair is on the HIP path")
    audio, sr = ref_audio
    if audio.ndim == 1:
        audio = audio[None]
    if audio.shape[0] > 1:
        audio = torch.mean(audio, dim=0, keepdim=True)
    rms = torch.sqrt(torch.mean(torch.square(audio)))
    if rms < target_rms:
        audio = audio * target_rms / rms
    if sr != target_sample_rate:
        audio = resample(audio, sr, target_sample_rate)
    device = device or getattr(model_obj, "device", None) or _default_device()
    audio = audio.to(device)

    if len(ref_text[-1].encode("utf-8")) == 1:
        ref_text = ref_text + " "

    def _infer_basic(gen_text):
        local_speed = 0.3 if len(gen_text.encode("utf-8")) < 10 else speed
        final_text_list = convert_char_to_pinyin([ref_text + gen_text])
        ref_audio_len = audio.shape[-1] // hop_length
        if fix_duration is not None:
            duration = int(fix_duration * target_sample_rate / hop_length)
        else:
            ref_text_len = len(ref_text.encode("utf-8"))
            gen_text_len = len(gen_text.encode("utf-8"))
            duration = ref_audio_len + int(ref_audio_len / ref_text_len * gen_text_len / local_speed)
        with torch.inference_mode():
            generated, _ = model_obj.sample(cond=audio, text=final_text_list, duration=duration, steps=nfe_step,
                                            cfg_strength=cfg_strength, sway_sampling_coef=sway_sampling_coef)
            del _
            generated = generated.to(torch.float32)[:, ref_audio_len:, :].permute(0, 2, 1)
            wav = vocoder.decode(generated)
            if rms < target_rms:
                wav = wav * rms / target_rms
            wav = wav.squeeze().cpu().numpy()
        return wav, generated

    it = (lambda xs: progress.tqdm(xs)) if progress is not None else (lambda xs: xs)
    if streaming:
        for gen_text in it(gen_text_batches):
            wav, generated = _infer_basic(gen_text)
            del generated
            for j in range(0, len(wav), chunk_size):
                yield wav[j: j + chunk_size], target_sample_rate
        return

    def _single(gen_text):
        wav, generated = _infer_basic(gen_text)
        return wav, generated[0].cpu().numpy()

    waves, specs = [], []
    with ThreadPoolExecutor() as ex:
        futures = [ex.submit(_single, t) for t in gen_text_batches]
        for fut in it(futures):
            res = fut.result()
            if res:
                waves.append(res[0])
                specs.append(res[1])
    if waves:
        yield cross_fade(waves, cross_fade_duration), target_sample_rate, np.concatenate(specs, axis=1)
    else:
        yield None, target_sample_rate, None
