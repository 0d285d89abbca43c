"""SIREN model and `fit_siren` — the MI355X drop-in for the reference hot path.

Reference: nerf_attention/siren.py.  `SineLayer` / `SIREN` (siren.py:17-67)
keep the reference's module tree, state_dict keys
(`network.{0..L}.linear.{weight,bias}`, `network.{L+1}.{weight,bias}`) and —
crucially for seeded parity — its exact CPU-RNG consumption order:
`nn.Linear.__init__` (kaiming_uniform_ weight, uniform_ bias), then the
SIREN re-draw of weight then bias.  Initialisation is the only RNG consumer
of a fit, so a fit started from the same torch seed starts from the same
parameters as the reference.

`fit_siren` (siren.py:70-149) keeps the reference signature and returns the
same `FitResult`, but the 2000-epoch loop runs on the HIP engine: two fused
kernels per epoch, no per-epoch host sync, metrics computed on the device.
There is no CPU fallback: a HIP request without a HIP device raises.  Only an
explicit device='cpu' (BASELINE config 1, `quickstart --cpu`) trains on the
host, in eager PyTorch (host_fit.py).
"""

from __future__ import annotations

import ctypes
import math

import numpy as np
import torch
import torch.nn as nn

from . import _native, engine
from .types import FitResult, SIRENConfig


class SineLayer(nn.Module):
    """y = sin(ω0 · (x Wᵀ + b)) — reference siren.py:17-34."""

    def __init__(self, in_features: int, out_features: int,
                 omega_0: float = 30.0, is_first: bool = False):
        super().__init__()
        self.omega_0 = omega_0
        # nn.Linear's own reset_parameters consumes the RNG first (as in the reference)
        self.linear = nn.Linear(in_features, out_features)
        if is_first:
            bound = 1.0 / in_features
        else:
            bound = math.sqrt(6.0 / in_features) / omega_0
        with torch.no_grad():
            self.linear.weight.uniform_(-bound, bound)
            self.linear.bias.uniform_(-bound, bound)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return torch.sin(self.omega_0 * self.linear(x))


class SIREN(nn.Module):
    """SineLayer(1, W, first) → L × SineLayer(W, W) → Linear(W, d) — siren.py:37-67."""

    def __init__(self, config: SIRENConfig, out_features: int):
        super().__init__()
        self.siren_config = config
        w, om = config.hidden_features, config.omega_0
        stack: list[nn.Module] = [SineLayer(1, w, omega_0=om, is_first=True)]
        stack += [SineLayer(w, w, omega_0=om) for _ in range(config.hidden_layers)]
        head = nn.Linear(w, out_features)
        bound = math.sqrt(6.0 / w) / om
        with torch.no_grad():
            head.weight.uniform_(-bound, bound)
            head.bias.uniform_(-bound, bound)
        stack.append(head)
        self.network = nn.Sequential(*stack)
        self.out_features = out_features

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        # Inference on a HIP device goes through the HIP forward kernel.  With
        # autograd recording (gradients wanted w.r.t. the parameters or the
        # positions x), on the CPU, or for a shape the engine does not take
        # (fewer than 2 positions, W/d_head/L outside the compiled set) the
        # module is plain torch, as the nn.Module it is.
        if x.is_cuda and self._engine_shape(x) and not (
                torch.is_grad_enabled() and
                (x.requires_grad or any(p.requires_grad for p in self.parameters()))):
            return self._native_forward(x)
        return self.network(x)

    def _engine_shape(self, x: torch.Tensor) -> bool:
        c = self.siren_config
        return (x.numel() >= 2 and (x.dim() == 1 or x.shape[-1] == 1)
                and c.hidden_features in (64, 128, 256, 512)
                and self.out_features in (64, 128) and 1 <= c.hidden_layers <= 4)

    def _native_forward(self, x: torch.Tensor) -> torch.Tensor:
        # The plan (device buffers + C-ABI descriptor) is cached across calls:
        # rebuilt when the position count or device changes, parameters
        # reloaded when any is replaced or modified in place (data_ptr /
        # _version).  Positions are copied in every call (N floats).
        pkey = tuple((p.data_ptr(), p._version) for p in self.parameters())
        xkey = (x.numel(), x.device)
        plan = self.__dict__.get('_fwd_plan')
        if plan is None or self._fwd_xkey != xkey:
            plan = engine.ForwardPlan(self.siren_config, self.out_features, x, 1, x.device)
            self._fwd_plan, self._fwd_xkey, self._fwd_pkey = plan, xkey, None
        else:
            plan.pos[:plan.n].copy_(x.reshape(-1))
        if self._fwd_pkey != pkey:
            plan.load(self.flat_parameters())
            self._fwd_pkey = pkey
        out = torch.empty(plan.y.shape, dtype=torch.float32, device=x.device)
        return plan(out)[0].to(x.dtype)

    def __getstate__(self):
        # the cached forward plan holds raw device pointers: never pickle it
        state = super().__getstate__() if hasattr(super(), '__getstate__') else self.__dict__
        return {k: v for k, v in state.items() if not k.startswith('_fwd_')}

    def flat_parameters(self) -> torch.Tensor:
        """All parameters concatenated in state_dict order (the engine's layout)."""
        return torch.cat([p.detach().reshape(-1) for p in self.state_dict().values()])

    @torch.no_grad()
    def load_flat_parameters(self, flat: torch.Tensor) -> None:
        off = 0
        for p in self.state_dict().values():
            n = p.numel()
            p.copy_(flat[off:off + n].view_as(p))
            off += n

    def count_parameters(self) -> int:
        return sum(p.numel() for p in self.parameters() if p.requires_grad)

    def size_bytes(self) -> int:
        return self.count_parameters() * 4


def _init_segments(config: SIRENConfig, out_features: int):
    """The uniform_ calls SIREN(config, out_features).__init__ makes, in order,
    as (count, bound, kept): per nn.Linear(in, out) its own reset
    (kaiming_uniform_ weight, uniform_ bias — overwritten, so only the draw
    count matters), then the SIREN re-draw of weight and bias in ±bound
    (siren.py:17-67; bounds as SineLayer / SIREN above compute them)."""
    w, om = config.hidden_features, config.omega_0
    linears = [(1, w, 1.0 / 1)]
    linears += [(w, w, math.sqrt(6.0 / w) / om)] * config.hidden_layers
    linears += [(w, out_features, math.sqrt(6.0 / w) / om)]
    segs = []
    for fan_in, fan_out, bound in linears:
        segs += [(fan_in * fan_out + fan_out, 0.0, False),
                 (fan_in * fan_out, bound, True), (fan_out, bound, True)]
    return segs


_STATE = slice(24, 24 + 624 * 8)   # CPUGeneratorImplState: u64 seed, i32 left, i32 seeded,
_LEFT, _SEEDED, _NEXT = slice(8, 12), slice(12, 16), slice(16, 24)   # u64 next, u64 state[624],
_STATE_BYTES = 5056                                                    # normal-sample cache


def _replay(segs) -> torch.Tensor | None:
    """Draw the segments (count, bound, kept) through the native replay of
    torch's default CPU generator, advancing it; None (and nothing drawn)
    when the generator state is not the CPUGeneratorImplState layout this
    replay reads (another torch build)."""
    counts = np.array([c for c, _b, _k in segs], dtype=np.int64)
    bounds = np.array([b for _c, b, _k in segs], dtype=np.float64)
    offs, off = np.full(len(segs), -1, dtype=np.int64), 0
    for i, (c, _b, kept) in enumerate(segs):
        if kept:
            offs[i], off = off, off + c
    raw = torch.get_rng_state().numpy().copy()
    if raw.size != _STATE_BYTES or raw[_SEEDED].view(np.int32)[0] != 1:
        return None
    flat = torch.empty(off, dtype=torch.float32)
    state = raw[_STATE].view(np.uint64).astype(np.uint32)
    left = ctypes.c_int32(int(raw[_LEFT].view(np.int32)[0]))
    nxt = ctypes.c_uint32(int(raw[_NEXT].view(np.uint64)[0]))
    lo = -bounds
    _native.check(_native.load().nerfhip_rng_uniform_segments(
        state.ctypes.data, ctypes.byref(left), ctypes.byref(nxt),
        len(segs), counts.ctypes.data, lo.ctypes.data, bounds.ctypes.data, offs.ctypes.data,
        flat.data_ptr()))
    raw[_STATE].view(np.uint64)[:] = state
    raw[_LEFT].view(np.int32)[0] = left.value
    raw[_NEXT].view(np.uint64)[0] = nxt.value
    torch.set_rng_state(torch.from_numpy(raw))
    return flat


_REPLAY_OK = None


def replay_matches_torch() -> bool:
    """One-time self-check of the native replay against torch's own uniform_
    on this host: the replay reproduces the rounding of torch's CPU kernel
    (x·span + lo contracted into one fma, as its AVX2 / AVX-512 paths do);
    under another kernel (ATEN_CPU_CAPABILITY=default, a host without FMA, a
    different torch) the bits could differ, and init_flat then builds the
    modules instead.  Shapes of SIREN layers: a discarded reset segment, a
    W x W weight, a bias, a short tail.  The caller's generator state is
    restored."""
    global _REPLAY_OK
    if _REPLAY_OK is None:
        probe = [(300, 0.0, False), (256 * 256, 0.05, True), (256, 0.05, True), (17, 1.0, True)]
        saved = torch.get_rng_state()
        try:
            torch.manual_seed(20240601)
            ref = [torch.empty(n).uniform_(-b, b) for n, b, _k in probe]
            torch.manual_seed(20240601)
            got = _replay(probe)
            _REPLAY_OK = got is not None and torch.equal(got, torch.cat(ref[1:]))
        finally:
            torch.set_rng_state(saved)
    return _REPLAY_OK


def init_flat(config: SIRENConfig, out_features: int) -> torch.Tensor:
    """The flat initial parameters `SIREN(config, out_features)` would hold
    (state_dict order), drawn from — and advancing — torch's default CPU
    generator exactly as that constructor does, without building the module:
    nerfhip_rng_uniform_segments replays torch's mt19937 + uniform_ on the
    host at the bare generator's speed (bit-identical, tests/test_host.py).
    The sweep's drivers use it to overlap the inits with training.  Where the
    replay cannot be shown to match torch's own kernel on this host
    (replay_matches_torch), or the generator state layout differs, it builds
    the module instead, which is exact by definition."""
    if replay_matches_torch():
        flat = _replay(_init_segments(config, out_features))
        if flat is not None:
            return flat
    return SIREN(config, out_features).flat_parameters()


def uninitialised(config: SIRENConfig, out_features: int, device) -> SIREN:
    """SIREN(config, out_features) on `device` with storage only — built on
    the meta device, so the constructor draws nothing from the generator —
    for parameters loaded right after (load_flat_parameters)."""
    with torch.device('meta'):
        m = SIREN(config, out_features)
    return m.to_empty(device=device)


def _finish(model: SIREN, config: SIRENConfig, out: engine.FitOutput, seq_len: int,
            d_head: int) -> FitResult:
    """FitResult exactly as siren.py:127-149 assembles it."""
    cos = torch.from_numpy(out.row_cos)
    raw_size = seq_len * d_head * 2
    siren_size = model.size_bytes()
    return FitResult(
        model=model,
        config=config,
        target_mean=out.target_mean,
        target_std=out.target_std,
        losses=out.losses,
        final_mse=out.final_mse,
        final_cosine_mean=cos.mean().item(),
        final_cosine_min=cos.min().item(),
        final_cosine_std=cos.std().item(),
        per_pos_mse=out.row_mse,
        cosine_sims=out.row_cos,
        compression_ratio=raw_size / siren_size,
        raw_size_bytes=raw_size,
        siren_size_bytes=siren_size,
        train_time_seconds=out.train_time_seconds,
        seq_len=seq_len,
        d_head=d_head,
        num_parameters=model.count_parameters(),
    )


def probe_line(epoch: int, epochs: int, norm_mse: float, real_mse: float, cos: float) -> str:
    """The verbose progress line of siren.py:112-115."""
    return (f"  Epoch {epoch}/{epochs} | "
            f"NormMSE: {norm_mse:.6f} | "
            f"RealMSE: {real_mse:.6f} | "
            f"CosSim: {cos:.4f}")


def fit_siren(
    kv_tensor: torch.Tensor,
    config: SIRENConfig,
    epochs: int = 5000,
    lr: float = 1e-4,
    device: str = 'cuda',
    log_every: int = 500,
    verbose: bool = True,
    *,
    precision: str | None = None,
) -> FitResult:
    """Fit a SIREN to one (seq_len, d_head) KV tensor on the MI355X engine.

    Same contract as the reference (siren.py:70-149): the input is not
    mutated, the torch CPU RNG is consumed exactly once (model init), the
    result owns its model (on `device`) and CPU copies of mean/std/metrics.
    Extension: `precision` ("bf16x3" default, or "fp32"; engine.PRECISIONS)
    picks the GEMM arithmetic — both meet the same per-fit parity bar.
    """
    seq_len, d_head = kv_tensor.shape
    if torch.device(device).type == 'cpu':
        # explicit host request (BASELINE config 1, quickstart --cpu): the
        # eager PyTorch loop, see host_fit.py.  Never reached for 'cuda'.
        from .host_fit import fit_on_host
        model = SIREN(config, out_features=d_head)
        show = (lambda e, n, r, c: print(probe_line(e, epochs, n, r, c))) if verbose else None
        return fit_on_host(kv_tensor, config, model, epochs, lr, log_every, show)
    dev = engine.resolve_device(device)
    model = SIREN(config, out_features=d_head)
    spec = engine.FitSpec(target=kv_tensor, config=config, init=model.flat_parameters())
    out = engine.run_fits([spec], epochs, lr=lr, log_every=log_every if verbose else 0,
                          devices=[dev.index], precision=precision)[0]
    model = model.to(dev)
    model.load_flat_parameters(out.params)
    model.eval()  # siren.py:119
    if verbose:
        for ep, nm, rm, cs in out.probes:
            print(probe_line(ep, epochs, nm, rm, cs))
    return _finish(model, config, out, seq_len, d_head)
