"""U-Net epsilon-predictor and Gaussian diffusion schedule — inference subset of the reference
red_diffeq/models/diffusion.py (Unet 220-301, blocks 78-218, schedules 304-326,
GaussianDiffusion 328-437, q_sample 516-519).

Module tree and parameter names are the reference's, so a reference checkpoint
(``torch.load(path)["model"]`` = a GaussianDiffusion state_dict, 296 keys at dim=64) loads
unchanged.  The RED regulariser only runs the forward pass (its U-Net output is detached,
regularization/diffusion.py:74), so training/sampling loops (p_losses, Trainer, Dataset,
ddim/p_sample loops) are out of scope.

The arithmetic of every block goes through ``red_diffeq.models.unet_ops``.
"""
import math
import os
from collections import namedtuple
from functools import partial

import torch
import torch.nn.functional as F
from torch import nn

from ..utils.diffusion_utils import extract
from . import unet_ops as ops

ModelPrediction = namedtuple("ModelPrediction", ["pred_noise", "pred_x_start"])


def exists(x):
    return x is not None


def default(val, d):
    if exists(val):
        return val
    return d() if callable(d) else d


def cast_tuple(t, length=1):
    return t if isinstance(t, tuple) else (t,) * length


def divisible_by(numer, denom):
    return numer % denom == 0


def identity(t, *args, **kwargs):
    return t


def normalize_to_neg_one_to_one(img):
    return img * 2 - 1


def unnormalize_to_zero_to_one(t):
    return (t + 1) * 0.5


class _Rearrange(nn.Module):
    """Parameter-free stand-in for einops' Rearrange at index 0 of Downsample (keeps keys); the
    pixel-unshuffle itself is folded into the following conv's gather (ops.UNSHUFFLE2)."""


def Upsample(dim, dim_out=None):
    """nearest x2 then 3x3 conv (reference diffusion.py:78-79); keys ``.1.weight/.1.bias``."""
    return nn.Sequential(nn.Upsample(scale_factor=2, mode="nearest"), nn.Conv2d(dim, default(dim_out, dim), 3, padding=1))


def Downsample(dim, dim_out=None):
    """2x2 pixel-unshuffle then 1x1 conv (reference diffusion.py:81-82)."""
    return nn.Sequential(_Rearrange(), nn.Conv2d(dim * 4, default(dim_out, dim), 1))


class RMSNorm(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.g = nn.Parameter(torch.ones(1, dim, 1, 1))

    def forward(self, x):
        return ops.rmsnorm(x, self.g)


class SinusoidalPosEmb(nn.Module):
    def __init__(self, dim, theta=10000):
        super().__init__()
        self.dim = dim
        self.theta = theta

    def forward(self, x):
        return ops.sinusoidal(x, self.dim, self.theta)


class Block(nn.Module):
    """conv3x3 -> GroupNorm(8) -> (scale+1, shift) -> SiLU (reference diffusion.py:134-149)."""

    def __init__(self, dim, dim_out, groups=8):
        super().__init__()
        self.proj = nn.Conv2d(dim, dim_out, 3, padding=1)
        self.norm = nn.GroupNorm(groups, dim_out)
        self.act = nn.SiLU()

    def forward(self, x, scale_shift=None, skip=None, post=None):
        """skip: the concatenated U-Net skip (293-299); post: added after the SiLU (the identity
        shortcut of ResnetBlock, 168)."""
        return ops.conv_group_norm_silu(x, self.proj, self.norm, scale_shift, skip=skip, post=post)


class ResnetBlock(nn.Module):
    def __init__(self, dim, dim_out, *, time_emb_dim=None, groups=8):
        super().__init__()
        self.mlp = nn.Sequential(nn.SiLU(), nn.Linear(time_emb_dim, dim_out * 2)) if exists(time_emb_dim) else None
        self.block1 = Block(dim, dim_out, groups=groups)
        self.block2 = Block(dim_out, dim_out, groups=groups)
        self.res_conv = nn.Conv2d(dim, dim_out, 1) if dim != dim_out else nn.Identity()

    def forward(self, x, time_emb=None, skip=None, scale_shift=None):
        """(reference 160-168); `skip` = the tensor the reference torch.cat's onto x first;
        `scale_shift` = this block's Linear(SiLU(time_emb)) when the caller formed it already."""
        if scale_shift is None and exists(self.mlp) and exists(time_emb):
            scale_shift = ops.linear(time_emb, self.mlp[1], act_in=1)   # Linear(SiLU(t)): (B, 2C)
        if isinstance(self.res_conv, nn.Conv2d):
            # block1's conv and the 1x1 shortcut in one launch; block2 adds the shortcut after its SiLU
            pair = ops.conv_group_norm_silu_shortcut(x, self.block1.proj, self.block1.norm, scale_shift, skip,
                                                     self.res_conv)
            if pair is not None:
                return self.block2(pair[0], post=pair[1])
            h = ops.block_pair(x, skip, self.block1, self.block2, scale_shift)   # bf16: one hand-off in bf16
            if h is None:
                h = self.block2(self.block1(x, scale_shift=scale_shift, skip=skip))
            return ops.conv2d(x, self.res_conv, x2=skip, residual=h)    # h + res_conv(x), fused
        if skip is None:
            h = ops.block_pair(x, None, self.block1, self.block2, scale_shift, post=x)
            if h is not None:
                return h
        h = self.block1(x, scale_shift=scale_shift, skip=skip)
        if skip is not None:
            x = torch.cat((x, skip), dim=1)
        return self.block2(h, post=x)                                    # h + x, fused


class LinearAttention(nn.Module):
    def __init__(self, dim, heads=4, dim_head=32, num_mem_kv=4):
        super().__init__()
        self.scale = dim_head ** -0.5
        self.heads = heads
        hidden = dim_head * heads
        self.norm = RMSNorm(dim)
        self.mem_kv = nn.Parameter(torch.randn(2, heads, dim_head, num_mem_kv))
        self.to_qkv = nn.Conv2d(dim, hidden * 3, 1, bias=False)
        self.to_out = nn.Sequential(nn.Conv2d(hidden, dim, 1), RMSNorm(dim))

    def forward(self, x):
        """Returns LinearAttention(x) + x (the residual of Unet.forward is fused)."""
        return ops.linear_attention(x, self)


class Attention(nn.Module):
    def __init__(self, dim, heads=4, dim_head=32, num_mem_kv=4, flash=False):
        super().__init__()
        self.heads = heads
        hidden = dim_head * heads
        self.norm = RMSNorm(dim)
        self.attend = nn.Identity()   # denoising-diffusion-pytorch Attend: no parameters
        self.mem_kv = nn.Parameter(torch.randn(2, heads, num_mem_kv, dim_head))
        self.to_qkv = nn.Conv2d(dim, hidden * 3, 1, bias=False)
        self.to_out = nn.Conv2d(hidden, dim, 1)

    def forward(self, x):
        """Returns Attention(x) + x (the residual of Unet.forward is fused)."""
        return ops.full_attention(x, self)


class Unet(nn.Module):
    """Same constructor and module tree as the reference Unet (diffusion.py:220-271)."""

    def __init__(self, dim, init_dim=None, out_dim=None, dim_mults=(1, 2, 4, 8), channels=3,
                 self_condition=False, resnet_block_groups=8, learned_variance=False,
                 learned_sinusoidal_cond=False, random_fourier_features=False, learned_sinusoidal_dim=16,
                 sinusoidal_pos_emb_theta=10000, attn_dim_head=32, attn_heads=4, full_attn=None,
                 flash_attn=False):
        super().__init__()
        if learned_sinusoidal_cond or random_fourier_features:
            raise NotImplementedError("learned/random Fourier time embeddings are not used by red-diffeq")
        self.channels = channels
        self.self_condition = self_condition
        input_channels = channels * (2 if self_condition else 1)
        init_dim = default(init_dim, dim)
        self.init_conv = nn.Conv2d(input_channels, init_dim, 7, padding=3)
        dims = [init_dim, *map(lambda m: dim * m, dim_mults)]
        in_out = list(zip(dims[:-1], dims[1:]))
        block = partial(ResnetBlock, groups=resnet_block_groups)
        time_dim = dim * 4
        self.random_or_learned_sinusoidal_cond = False
        self.time_mlp = nn.Sequential(SinusoidalPosEmb(dim, theta=sinusoidal_pos_emb_theta),
                                      nn.Linear(dim, time_dim), nn.GELU(), nn.Linear(time_dim, time_dim))
        if not full_attn:
            full_attn = (*((False,) * (len(dim_mults) - 1)), True)
        n = len(dim_mults)
        full_attn = cast_tuple(full_attn, n)
        attn_heads = cast_tuple(attn_heads, n)
        attn_dim_head = cast_tuple(attn_dim_head, n)
        self.downs = nn.ModuleList([])
        self.ups = nn.ModuleList([])
        for ind, ((di, do), fa, hh, dh) in enumerate(zip(in_out, full_attn, attn_heads, attn_dim_head)):
            last = ind >= len(in_out) - 1
            attn = Attention if fa else LinearAttention
            self.downs.append(nn.ModuleList([
                block(di, di, time_emb_dim=time_dim), block(di, di, time_emb_dim=time_dim),
                attn(di, dim_head=dh, heads=hh),
                Downsample(di, do) if not last else nn.Conv2d(di, do, 3, padding=1)]))
        mid = dims[-1]
        self.mid_block1 = block(mid, mid, time_emb_dim=time_dim)
        self.mid_attn = Attention(mid, heads=attn_heads[-1], dim_head=attn_dim_head[-1])
        self.mid_block2 = block(mid, mid, time_emb_dim=time_dim)
        for ind, ((di, do), fa, hh, dh) in enumerate(zip(*map(reversed, (in_out, full_attn, attn_heads, attn_dim_head)))):
            last = ind == len(in_out) - 1
            attn = Attention if fa else LinearAttention
            self.ups.append(nn.ModuleList([
                block(do + di, do, time_emb_dim=time_dim), block(do + di, do, time_emb_dim=time_dim),
                attn(do, dim_head=dh, heads=hh),
                Upsample(do, di) if not last else nn.Conv2d(do, di, 3, padding=1)]))
        self.out_dim = default(out_dim, channels * (1 if not learned_variance else 2))
        self.final_res_block = block(dim * 2, dim, time_emb_dim=time_dim)
        self.final_conv = nn.Conv2d(dim, self.out_dim, 1)
        self.precision = "fp32"     # conv arithmetic: "fp32" (reference) or "bf16" (configs[4])

    def set_precision(self, mode):
        """U-Net convolutions in "fp32" (the reference's arithmetic, default) or "bf16" (bf16
        operands, fp32 accumulation; new behaviour for large tiled models, configs[4])."""
        with ops.precision(mode):
            pass
        self.precision = mode
        return self

    @property
    def downsample_factor(self):
        return 2 ** (len(self.downs) - 1)

    def _time(self, time):
        return ops.time_mlp(time, self.time_mlp)                          # one launch

    def _resnet_blocks(self):
        """The ResnetBlocks in forward order."""
        bl = [b for b1, b2, _, _ in self.downs for b in (b1, b2)] + [self.mid_block1, self.mid_block2]
        return bl + [b for b1, b2, _, _ in self.ups for b in (b1, b2)] + [self.final_res_block]

    def _resample(self, x, m):
        if isinstance(m, nn.Conv2d):
            return ops.conv2d(x, m)
        if isinstance(m[0], nn.Upsample):
            return ops.conv2d(x, m[1], mode=ops.UPSAMPLE2)               # nearest x2 folded in
        return ops.conv2d(x, m[1], mode=ops.UNSHUFFLE2)                  # pixel-unshuffle folded in

    # Small no-grad forwards (the RED regulariser's per-iteration call, B = 1..16 at 72 x 72) are
    # launch-bound: ~150 kernels of a few microseconds.  They are captured once per (shape,
    # precision, weights version) into a hipGraph and replayed (RDQ_NO_UNET_GRAPH=1 disables).
    GRAPH_MAX_PIXELS = 16 * 72 * 72

    def forward(self, x, time, x_self_cond=None):
        assert all(divisible_by(d, self.downsample_factor) for d in x.shape[-2:]), \
            f"your input dimensions {x.shape[-2:]} need to be divisible by {self.downsample_factor}, given the unet"
        if (x.is_cuda and not torch.is_grad_enabled() and x_self_cond is None and not self.self_condition
                and x.shape[0] * x.shape[2] * x.shape[3] <= self.GRAPH_MAX_PIXELS
                and not os.environ.get("RDQ_NO_UNET_GRAPH")
                and not torch.cuda.is_current_stream_capturing()):
            return self._graphed(x, time)
        with ops.precision(self.precision):
            return self._forward(x, time, x_self_cond)

    def _apply(self, fn, *args, **kwargs):
        # .to() / .cuda() / .float() may move or replace the parameters: captured graphs hold the
        # old addresses, so bump the weights generation (the graph cache key)
        self._wgen = getattr(self, "_wgen", 0) + 1
        return super()._apply(fn, *args, **kwargs)

    def _weights_version(self):
        """Graph-cache key of the weights.  A replay reads the parameters' storage at the addresses
        captured, so the key holds every parameter's data_ptr: a parameter replaced without _apply
        (load_state_dict(assign=True), ``p.data = t``, a new nn.Parameter on a submodule) changes it
        and forces a recapture.  In-place updates (optimizer steps, load_state_dict
        copies) keep the addresses and need none in fp32; the bf16 path reads packed copies, so
        there the parameters' version counters are part of the key too.  So is the library's kernel-option
        generation (rdq_unet_options_generation): graphs captured under other options are recaptured."""
        ptrs = tuple(p.data_ptr() for p in self.parameters())
        # kernel options (rdq_unet_set_option) choose kernels at capture time: a change recaptures
        from .. import _hip
        opt = int(_hip.lib().rdq_unet_options_generation())
        if self.precision == "bf16":
            return (getattr(self, "_wgen", 0), opt, ptrs, tuple(p._version for p in self.parameters()))
        return (getattr(self, "_wgen", 0), opt, ptrs)

    def _graphed(self, x, time):
        ent = self._graph_entry(x, time)
        ent["x"].copy_(x)
        ent["t"].copy_(time)
        ent["graph"].replay()
        return ent["y"].clone()

    def graph_io(self, shape, device, time_dtype=torch.int64):
        """The static (x, t) input buffers of the captured no-grad forward for inputs of `shape` (None
        where forward() would not replay a graph).  A caller that writes its inputs straight into them
        (ops.red_q_sample_into, the RED regulariser) and calls replay_static() pays neither the input
        copies nor the output clone of forward()."""
        B, _, H, W = shape
        if (torch.device(device).type != "cuda" or torch.is_grad_enabled() or self.self_condition
                or B * H * W > self.GRAPH_MAX_PIXELS or os.environ.get("RDQ_NO_UNET_GRAPH")
                or torch.cuda.is_current_stream_capturing()):
            return None
        device = torch.device(device)
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        ent = self.__dict__.get("_graphs", {}).get(
            (tuple(shape), torch.float32, device, self.precision, time_dtype))
        if ent is None or ent["ver"] != self._weights_version():      # capture once, on placeholders
            ent = self._graph_entry(torch.zeros(shape, device=device, dtype=torch.float32),
                                    torch.zeros(B, device=device, dtype=time_dtype))
        return ent["x"], ent["t"]

    def replay_static(self, xs, ts):
        """Replay the forward captured for the static buffers (xs, ts) of graph_io; returns the static
        output (overwritten by the next replay of the same shape)."""
        ent = self.__dict__.get("_graphs", {}).get((tuple(xs.shape), xs.dtype, xs.device, self.precision, ts.dtype))
        if ent is None or ent["x"] is not xs or ent["t"] is not ts:
            raise RuntimeError("replay_static: (xs, ts) are not the static inputs of a captured forward (graph_io)")
        ent["graph"].replay()
        return ent["y"]

    def _graph_entry(self, x, time):
        """The captured forward for x's shape and time's dtype (captured now, on copies of x / time as its
        static inputs, if missing or stale)."""
        key = (tuple(x.shape), x.dtype, x.device, self.precision, time.dtype)
        cache = self.__dict__.setdefault("_graphs", {})
        ver = self._weights_version()
        ent = cache.get(key)
        if ent is None or ent["ver"] != ver:
            xs, ts = x.detach().clone(), time.detach().clone()
            side = torch.cuda.Stream(device=x.device)
            side.wait_stream(torch.cuda.current_stream(x.device))
            with torch.cuda.stream(side), ops.precision(self.precision):
                self._forward(xs, ts, None)            # warm-up: weight packs, workspaces, code objects
            torch.cuda.current_stream(x.device).wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph), ops.precision(self.precision):
                ys = self._forward(xs, ts, None)
            ent = {"ver": ver, "graph": graph, "x": xs, "t": ts, "y": ys}
            cache[key] = ent
        return ent

    def _forward(self, x, time, x_self_cond):
        if self.self_condition:
            x_self_cond = default(x_self_cond, lambda: torch.zeros_like(x))
            x = torch.cat((x_self_cond, x), dim=1)
        x, t = ops.head(x, self.init_conv, time, self.time_mlp)          # init_conv + time_mlp: one launch
        r = x
        blocks = self._resnet_blocks()
        first = ops.first_block_and_scale_shifts(x, self.downs[0][0], t, blocks)
        if first is None:
            ss = iter(ops.resnet_scale_shifts(t, blocks))                 # all blocks' Linear(SiLU(t))
        else:
            ss = iter(first[1])                 # formed in the first block's conv launch
        h = []
        for i, (b1, b2, attn, down) in enumerate(self.downs):
            if i == 0 and first is not None:
                x = first[0]
                next(ss)
            else:
                x = b1(x, t, scale_shift=next(ss))
            h.append(x)
            x = b2(x, t, scale_shift=next(ss))
            x = attn(x)                       # attn(x) + x
            h.append(x)
            x = self._resample(x, down)
        x = self.mid_block1(x, t, scale_shift=next(ss))
        x = self.mid_attn(x)
        x = self.mid_block2(x, t, scale_shift=next(ss))
        for b1, b2, attn, up in self.ups:
            x = b1(x, t, skip=h.pop(), scale_shift=next(ss))   # cat((x, skip)) folded into the conv gather
            x = b2(x, t, skip=h.pop(), scale_shift=next(ss))
            x = attn(x)
            x = self._resample(x, up)
        ss_last = next(ss)
        out = ops.last_block_and_out(x, self.final_res_block, ss_last, r, self.final_conv)
        if out is not None:
            return out                          # final_res_block's last pass feeds final_conv
        x = self.final_res_block(x, t, skip=r, scale_shift=ss_last)
        return ops.conv2d(x, self.final_conv)


# ------------------------------------------------------------------------------ schedules
def linear_beta_schedule(timesteps):
    scale = 1000 / timesteps
    return torch.linspace(scale * 0.0001, scale * 0.02, timesteps, dtype=torch.float64)


def cosine_beta_schedule(timesteps, s=0.008):
    steps = timesteps + 1
    t = torch.linspace(0, timesteps, steps, dtype=torch.float64) / timesteps
    ac = torch.cos((t + s) / (1 + s) * math.pi * 0.5) ** 2
    ac = ac / ac[0]
    return torch.clip(1 - ac[1:] / ac[:-1], 0, 0.999)


def sigmoid_beta_schedule(timesteps, start=-3, end=3, tau=1, clamp_min=1e-05):
    steps = timesteps + 1
    t = torch.linspace(0, timesteps, steps, dtype=torch.float64) / timesteps
    v_start = torch.tensor(start / tau).sigmoid()
    v_end = torch.tensor(end / tau).sigmoid()
    ac = (-((t * (end - start) + start) / tau).sigmoid() + v_end) / (v_end - v_start)
    ac = ac / ac[0]
    return torch.clip(1 - ac[1:] / ac[:-1], 0, 0.999)


class GaussianDiffusion(nn.Module):
    """Schedule buffers + the inference-side q/p math (reference diffusion.py:328-437, 516-519)."""

    def __init__(self, model, *, image_size, timesteps=1000, sampling_timesteps=None, objective="pred_v",
                 beta_schedule="sigmoid", schedule_fn_kwargs=dict(), ddim_sampling_eta=0.0,
                 auto_normalize=True, offset_noise_strength=0.0, min_snr_loss_weight=False, min_snr_gamma=5):
        super().__init__()
        assert not (type(self) == GaussianDiffusion and model.channels != model.out_dim)
        self.model = model
        self.channels = model.channels
        self.self_condition = model.self_condition
        if isinstance(image_size, int):
            image_size = (image_size, image_size)
        assert isinstance(image_size, (tuple, list)) and len(image_size) == 2
        self.image_size = image_size
        assert objective in {"pred_noise", "pred_x0", "pred_v"}
        self.objective = objective
        fn = {"linear": linear_beta_schedule, "cosine": cosine_beta_schedule,
              "sigmoid": sigmoid_beta_schedule}.get(beta_schedule)
        if fn is None:
            raise ValueError(f"unknown beta schedule {beta_schedule}")
        betas = fn(timesteps, **schedule_fn_kwargs)
        alphas = 1.0 - betas
        ac = torch.cumprod(alphas, dim=0)
        ac_prev = F.pad(ac[:-1], (1, 0), value=1.0)
        self.num_timesteps = int(betas.shape[0])
        self.sampling_timesteps = default(sampling_timesteps, self.num_timesteps)
        assert self.sampling_timesteps <= self.num_timesteps
        self.is_ddim_sampling = self.sampling_timesteps < self.num_timesteps
        self.ddim_sampling_eta = ddim_sampling_eta
        reg = lambda name, val: self.register_buffer(name, val.to(torch.float32))  # noqa: E731
        reg("betas", betas)
        reg("alphas_cumprod", ac)
        reg("alphas_cumprod_prev", ac_prev)
        reg("sqrt_alphas_cumprod", torch.sqrt(ac))
        reg("sqrt_one_minus_alphas_cumprod", torch.sqrt(1.0 - ac))
        reg("log_one_minus_alphas_cumprod", torch.log(1.0 - ac))
        reg("sqrt_recip_alphas_cumprod", torch.sqrt(1.0 / ac))
        reg("sqrt_recipm1_alphas_cumprod", torch.sqrt(1.0 / ac - 1))
        pv = betas * (1.0 - ac_prev) / (1.0 - ac)
        reg("posterior_variance", pv)
        reg("posterior_log_variance_clipped", torch.log(pv.clamp(min=1e-20)))
        reg("posterior_mean_coef1", betas * torch.sqrt(ac_prev) / (1.0 - ac))
        reg("posterior_mean_coef2", (1.0 - ac_prev) * torch.sqrt(alphas) / (1.0 - ac))
        self.offset_noise_strength = offset_noise_strength
        snr = ac / (1 - ac)
        clipped = snr.clone()
        if min_snr_loss_weight:
            clipped.clamp_(max=min_snr_gamma)
        if objective == "pred_noise":
            reg("loss_weight", clipped / snr)
        elif objective == "pred_x0":
            reg("loss_weight", clipped)
        else:
            reg("loss_weight", clipped / (snr + 1))
        self.normalize = normalize_to_neg_one_to_one if auto_normalize else identity
        self.unnormalize = unnormalize_to_zero_to_one if auto_normalize else identity

    @property
    def device(self):
        return self.betas.device

    def predict_start_from_noise(self, x_t, t, noise):
        return extract(self.sqrt_recip_alphas_cumprod, t, x_t.shape) * x_t - \
            extract(self.sqrt_recipm1_alphas_cumprod, t, x_t.shape) * noise

    def predict_noise_from_start(self, x_t, t, x0):
        return (extract(self.sqrt_recip_alphas_cumprod, t, x_t.shape) * x_t - x0) / \
            extract(self.sqrt_recipm1_alphas_cumprod, t, x_t.shape)

    def predict_v(self, x_start, t, noise):
        return extract(self.sqrt_alphas_cumprod, t, x_start.shape) * noise - \
            extract(self.sqrt_one_minus_alphas_cumprod, t, x_start.shape) * x_start

    def predict_start_from_v(self, x_t, t, v):
        return extract(self.sqrt_alphas_cumprod, t, x_t.shape) * x_t - \
            extract(self.sqrt_one_minus_alphas_cumprod, t, x_t.shape) * v

    def q_posterior(self, x_start, x_t, t):
        mean = extract(self.posterior_mean_coef1, t, x_t.shape) * x_start + \
            extract(self.posterior_mean_coef2, t, x_t.shape) * x_t
        return (mean, extract(self.posterior_variance, t, x_t.shape),
                extract(self.posterior_log_variance_clipped, t, x_t.shape))

    def model_predictions(self, x, t, x_self_cond=None, clip_x_start=False, rederive_pred_noise=False):
        out = self.model(x, t, x_self_cond)
        clip = partial(torch.clamp, min=-1.0, max=1.0) if clip_x_start else identity
        if self.objective == "pred_noise":
            pred_noise = out
            x_start = clip(self.predict_start_from_noise(x, t, pred_noise))
            if clip_x_start and rederive_pred_noise:
                pred_noise = self.predict_noise_from_start(x, t, x_start)
        elif self.objective == "pred_x0":
            x_start = clip(out)
            pred_noise = self.predict_noise_from_start(x, t, x_start)
        else:
            x_start = clip(self.predict_start_from_v(x, t, out))
            pred_noise = self.predict_noise_from_start(x, t, x_start)
        return ModelPrediction(pred_noise, x_start)

    def p_mean_variance(self, x, t, x_self_cond=None, clip_denoised=True):
        preds = self.model_predictions(x, t, x_self_cond)
        x_start = preds.pred_x_start
        if clip_denoised:
            x_start.clamp_(-1.0, 1.0)
        mean, var, logvar = self.q_posterior(x_start=x_start, x_t=x, t=t)
        return mean, var, logvar, x_start

    def p_sample_deterministic(self, x, t: int, x_self_cond=None):
        bt = torch.full((x.shape[0],), t, device=x.device, dtype=torch.long)
        mean, _, _, x_start = self.p_mean_variance(x=x, t=bt, x_self_cond=x_self_cond, clip_denoised=True)
        return mean, x_start

    def q_sample(self, x_start, t, noise=None):
        noise = default(noise, lambda: torch.randn_like(x_start))
        return extract(self.sqrt_alphas_cumprod, t, x_start.shape) * x_start + \
            extract(self.sqrt_one_minus_alphas_cumprod, t, x_start.shape) * noise
