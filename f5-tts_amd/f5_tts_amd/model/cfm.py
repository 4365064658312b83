"""Engine-backed conditional flow matching sampler: a drop-in `model_obj` for
`infer_process` / `F5TTS.ema_model` / eval drivers.

`CFM.sample` keeps the reference signature and return tuple (`cfm.py:83-102,229`). The host
preamble (mel intake, tokenisation, duration rule, cond padding/masks, noise recipe, time
grid) is restated here in PyTorch exactly as `cfm.py:105-216` does it; the ODE loop, the
backbone forwards, CFG, the Euler update and the final cond overwrite run in the HIP
engine (`f5h_sample`, include/f5h.h). There is no PyTorch fallback for the loop.
"""

from __future__ import annotations

from typing import Callable

import torch
import torch.nn.functional as F
from torch import nn
from torch.nn.utils.rnn import pad_sequence

from .utils import default, exists, lens_to_mask, list_str_to_idx, list_str_to_tensor, time_grid


def _host_ints(x, batch):
    """Python ints of a host-side length argument (int, list/tuple, CPU tensor), or None if on a device."""
    if isinstance(x, int):
        return [x] * batch
    if isinstance(x, (list, tuple)):
        return [int(v) for v in x]
    if torch.is_tensor(x) and x.device.type == "cpu":
        v = [int(a) for a in x.reshape(-1).tolist()]
        return v * batch if len(v) == 1 else v
    return None


def _duration_rule_on_host(text, duration, lens, batch, cond_seq_len, max_duration):
    """duration = clamp(max(max(#tokens, lens) + 1, duration), max_duration) (cfm.py:135-139) from host
    values: exact whenever the token counts are on the host, and also for device-resident text when every
    requested duration already exceeds the padded text width (#tokens <= text.shape[1]) and the prompt."""
    dur = _host_ints(duration, batch)
    ln = [cond_seq_len] * batch if lens is None else _host_ints(lens, batch)
    if dur is None or ln is None or len(dur) != batch or len(ln) != batch:
        return None
    if text.device.type == "cpu":
        ntok = (text != -1).sum(dim=-1).tolist()
    elif all(d >= max(text.shape[1], lv) + 1 for d, lv in zip(dur, ln)):
        ntok = [0] * batch  # the requested durations dominate whatever the counts are
    else:
        return None
    return [min(max(max(int(t), lv) + 1, d), int(max_duration)) for t, lv, d in zip(ntok, ln, dur)]


def _to_device(vals, device):
    """Small host int list -> device LongTensor without a stream sync (pinned, non-blocking copy)."""
    t = torch.tensor(vals, dtype=torch.long)
    if torch.device(device).type == "cuda":
        return t.pin_memory().to(device, non_blocking=True)
    return t.to(device)


class CFM(nn.Module):
    def __init__(self, transformer: nn.Module, sigma=0.0, odeint_kwargs: dict = dict(method="euler"),
                 audio_drop_prob=0.3, cond_drop_prob=0.2, num_channels=None, mel_spec_module: nn.Module | None = None,
                 mel_spec_kwargs: dict = dict(), frac_lengths_mask=(0.7, 1.0), vocab_char_map: dict | None = None,
                 compute: str = "auto"):
        super().__init__()
        if odeint_kwargs.get("method", "euler") != "euler":
            raise NotImplementedError("the engine integrates with fixed-grid Euler (the reference default, "
                                      "utils_infer.py:62 ode_method='euler')")
        self.frac_lengths_mask = frac_lengths_mask
        if mel_spec_module is None:
            from ..mel import MelSpec

            mel_spec_module = MelSpec(**mel_spec_kwargs)
        self.mel_spec = mel_spec_module
        self.num_channels = default(num_channels, getattr(self.mel_spec, "n_mel_channels", 100))
        self.audio_drop_prob = audio_drop_prob
        self.cond_drop_prob = cond_drop_prob
        self.transformer = transformer
        self.dim = transformer.dim
        self.sigma = sigma
        self.odeint_kwargs = odeint_kwargs
        self.vocab_char_map = vocab_char_map
        if compute not in ("auto", "fp32", "bf16", "fp16"):
            raise ValueError(f"compute must be 'auto', 'fp32', 'bf16' or 'fp16', got {compute!r}")
        self.compute = compute

    @property
    def device(self):
        return next(self.parameters()).device

    def engine_compute(self) -> str:
        """"auto": the parameter dtype picks the mode (fp32 -> parity, fp16 -> fp16 MFMA as the reference
        runs on GPUs, utils_infer.py:190-199; bf16 -> bf16 MFMA); or "fp32" / "bf16" / "fp16" explicitly."""
        if self.compute != "auto":
            return self.compute
        from .backbones.base import compute_for_dtype

        return compute_for_dtype(next(self.parameters()).dtype)

    @torch.no_grad()
    def sample(self, cond, text, duration, *, lens=None, steps=32, cfg_strength=1.0, sway_sampling_coef=None,
               seed: int | None = None, max_duration=65536, vocoder: Callable | None = None, use_epss=True,
               no_ref_audio=False, duplicate_test=False, t_inter=0.1, edit_mask=None, y0=None,
               keep_trajectory: bool = True):
        """Same arguments/returns as the reference `CFM.sample`; extra keyword `y0` supplies the
        initial noise explicitly (parity tests), `keep_trajectory=False` skips the [steps+1,...] copy."""
        if self.training:
            self.eval()
        pdtype = next(self.parameters()).dtype
        if cond.ndim == 2:  # raw wave -> mel (cfm.py:106-109)
            cond = self.mel_spec(cond)
            cond = cond.permute(0, 2, 1)
            assert cond.shape[-1] == self.num_channels
        cond = cond.to(pdtype)
        batch, cond_seq_len, device = *cond.shape[:2], cond.device

        if isinstance(text, list):
            if exists(self.vocab_char_map):
                text = list_str_to_idx(text, self.vocab_char_map)
            else:
                text = list_str_to_tensor(text)
            assert text.shape[0] == batch

        # The duration rule (cfm.py:132-139) decides the padded length, which the host needs. When the
        # lengths are host values (ints, lists, CPU tensors) it is evaluated on the host and nothing waits
        # for the device, so back-to-back calls keep the GPU busy; device-resident lengths take one sync.
        dur_host = _duration_rule_on_host(text, duration, lens, batch, cond_seq_len, max_duration)
        if dur_host is not None:
            lens_host = [cond_seq_len] * batch if lens is None else _host_ints(lens, batch)
            lens = _to_device(lens_host, device)
            duration = _to_device(dur_host, device)
            if text.device.type == "cpu" and torch.device(device).type == "cuda":
                text = text.pin_memory().to(device, non_blocking=True)
            else:
                text = text.to(device)
        else:
            text = text.to(device)
            if not exists(lens):
                lens = torch.full((batch,), cond_seq_len, device=device, dtype=torch.long)
            lens = lens.to(device)
            if isinstance(duration, int):
                duration = torch.full((batch,), duration, device=device, dtype=torch.long)
            duration = torch.as_tensor(duration).to(device)
            duration = torch.maximum(torch.maximum((text != -1).sum(dim=-1), lens) + 1, duration)
            duration = duration.clamp(max=max_duration)
            dur_host = [int(d) for d in duration.tolist()]  # the one host sync of this path
        max_duration = max(dur_host)
        if edit_mask is not None:
            cond_mask = lens_to_mask(lens) & edit_mask
        else:  # == F.pad(lens_to_mask(lens), ...) below: max_duration > lens.amax() by the rule above
            cond_mask = lens_to_mask(lens, length=max_duration)

        if duplicate_test:  # inner-time-step observation corner (cfm.py:141-143)
            test_cond = F.pad(cond, (0, 0, cond_seq_len, max_duration - 2 * cond_seq_len), value=0.0)

        cond = F.pad(cond, (0, 0, 0, max_duration - cond_seq_len), value=0.0)
        if no_ref_audio:
            cond = torch.zeros_like(cond)
        cond_mask = F.pad(cond_mask, (0, max_duration - cond_mask.shape[-1]), value=False)
        use_batch_mask = batch > 1  # cfm.py:155-158

        if y0 is None:  # noise recipe of cfm.py:196-201 (per utterance, same seed each)
            ys = []
            for dur in dur_host:
                if exists(seed):
                    torch.manual_seed(seed)
                ys.append(torch.randn(dur, self.num_channels, device=self.device, dtype=pdtype))
            y0 = pad_sequence(ys, padding_value=0, batch_first=True)

        t_start = 0.0
        if duplicate_test:  # cfm.py:205-209
            t_start = t_inter
            y0 = (1 - t_start) * y0 + t_start * test_cond
            steps = int(steps * (1 - t_start))

        # the grid is a host constant of the call: built on the CPU in the parameter dtype (cfm.py:211-216)
        t = time_grid(steps, sway_sampling_coef, use_epss, device="cpu", dtype=pdtype, t_start=t_start)
        t_host = t.float().numpy()

        eng = self.transformer.get_engine(self.engine_compute(), self.device)
        out, traj = eng.sample(cond.float(), cond_mask, text, duration, y0.float(), t_host, float(cfg_strength),
                               use_batch_mask, keep_trajectory=keep_trajectory)
        out = out.to(pdtype)
        if traj is not None:
            traj = traj.to(pdtype)
        if exists(vocoder):
            out = vocoder(out.permute(0, 2, 1))
        return out, traj

    def forward(self, *args, **kwargs):
        raise NotImplementedError("training (CFM.forward, cfm.py:231-302) is out of scope for the sampling engine")
