"""f5_tts_amd — MI355X-native (gfx950) CFM sampling engine for F5-TTS / E2-TTS.

The reference's `CFM.sample()` ODE loop and its DiT/UNetT forward run as hand-written
HIP kernels (libf5h.so, C ABI in include/f5h.h); this package is the host-side mirror of
the reference's Python surface (`f5_tts.model.{CFM, DiT, UNetT}`, `f5_tts.api.F5TTS`).
"""

__version__ = "0.1.0"


def release_memory() -> int:
    """Wait for queued engine / Vocos / log-mel releases, then return the device pool's unused memory to the
    system (f5h_release_pending(2); waits for the device). Returns the releases still pending (0)."""
    from . import _lib

    return int(_lib.lib().f5h_release_pending(2))
