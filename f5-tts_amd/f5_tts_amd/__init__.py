"""f5_tts_amd — MI355X-native (gfx950) CFM sampling engine for F5-TTS / E2-TTS.

The reference's `CFM.sample()` ODE loop and its DiT/UNetT forward run as hand-written
HIP kernels (libf5h.so, C ABI in include/f5h.h); this package is the host-side mirror of
the reference's Python surface (`f5_tts.model.{CFM, DiT, UNetT}`, `f5_tts.api.F5TTS`).
"""

__version__ = "0.1.0"
