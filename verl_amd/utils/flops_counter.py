"""Model-FLOPs-utilisation bookkeeping of the update RPCs (verl/utils/flops_counter.py:32-241).

``perf/mfu/actor`` and ``perf/mfu/critic`` (fsdp_workers.py:690-694, 1247-1249) divide the model
FLOPs of one update by the time it took and by the device's promised dense rate. The reference's
device table stops at MI300X (flops_counter.py:46-47); this one knows the MI350-series parts
(dense bf16 MFMA: MI355X ~2.5 PF/s, MI350X ~2.3 PF/s; /opt/skills MI355X_MICROARCH.md, not the
2:1-sparsity figures). Unknown devices promise infinity, as the reference's do, so their MFU is 0.

FLOPs per token follow the reference's accounting: 6 x (dense weights touched per token) for
forward + backward, plus 12 x sum(seqlen^2) x head_dim x heads x layers for attention
(no causal halving), with the lm_head and the embedding both counted (2 x V x H).
"""

from __future__ import annotations

import torch

# dense bf16 / fp16 matrix peak per device name substring, FLOP/s (first match wins)
_DEVICE_FLOPS = (
    ("MI355X", 2.5e15),
    ("MI350X", 2.3e15),
    ("MI325X", 1307.4e12),
    ("MI300X", 1336e12),
    ("H100", 989e12),
    ("H800", 989e12),
    ("H200", 989e12),
    ("A100", 312e12),
    ("A800", 312e12),
)

_UNITS = {"B": 1.0, "K": 1e3, "M": 1e6, "G": 1e9, "T": 1e12, "P": 1e15}

VALID_CONFIG_TYPE = {"llama", "qwen2", "qwen2_vl", "qwen2_5_vl", "qwen3", "qwen2_moe", "qwen3_moe"}


# by ISA when the marketing name is missing (ROCm reports "AMD Radeon Graphics" without the
# amdgpu.ids table): gfx950 = MI350 series, taken as the MI355X of this deployment; gfx942 = MI300X
_ARCH_FLOPS = (("gfx950", 2.5e15), ("gfx942", 1336e12))


def _device_name() -> str:
    if not torch.cuda.is_available():
        return ""
    name = torch.cuda.get_device_name()
    if not any(key in name for key, _ in _DEVICE_FLOPS):
        name = f"{name} {getattr(torch.cuda.get_device_properties(0), 'gcnArchName', '')}"
    return name


def get_device_flops(unit: str = "T", device_name: str | None = None) -> float:
    """Promised dense bf16 FLOP/s of this device in ``unit`` (float('inf') when unknown)."""
    if device_name is None:
        device_name = _device_name()
    for key, flops in _DEVICE_FLOPS + _ARCH_FLOPS:
        if key in device_name:
            return flops / _UNITS[unit]
    return float("inf")


def _text_config(config):
    """Decoder dimensions live in ``text_config`` for the VL families (Qwen2-VL)."""
    return getattr(config, "text_config", None) or config


class FlopsCounter:
    """flops_counter.py:66-241: ``estimate_flops(batch_seqlens, delta_time) -> (achieved TFLOP/s,
    promised TFLOP/s)``; achieved is 0 for model types it does not know."""

    def __init__(self, config, device_name: str | None = None):
        self.config = config
        self.model_type = getattr(config, "model_type", "")
        self.device_name = device_name
        if self.model_type not in VALID_CONFIG_TYPE:
            print(f"Only support config type of {VALID_CONFIG_TYPE}, but got {self.model_type}. MFU will always be zero.")

    def _dense_params_per_token(self) -> float:
        c = _text_config(self.config)
        h = c.hidden_size
        heads = c.num_attention_heads
        d = getattr(c, "head_dim", None) or h // heads
        attn = h * d * (2 * heads + 2 * c.num_key_value_heads)  # q, o and k, v projections
        if self.model_type in ("qwen2_moe", "qwen3_moe"):
            mlp = h * c.moe_intermediate_size * 3 * c.num_experts_per_tok + h * c.num_experts
        else:
            mlp = 3 * h * c.intermediate_size  # gate, up, down (SwiGLU)
        return (attn + mlp) * c.num_hidden_layers + 2 * c.vocab_size * h

    def _attention_flops(self, batch_seqlens) -> float:
        c = _text_config(self.config)
        heads = c.num_attention_heads
        d = getattr(c, "head_dim", None) or c.hidden_size // heads
        sq = sum(int(s) * int(s) for s in batch_seqlens)
        return 12.0 * sq * d * heads * c.num_hidden_layers

    def estimate_flops(self, batch_seqlens, delta_time: float):
        """batch_seqlens: valid tokens of every sequence of the update (meta_info
        global_token_num); delta_time: seconds. Returns TFLOP/s (achieved, promised)."""
        promised = get_device_flops("T", self.device_name)
        if self.model_type not in VALID_CONFIG_TYPE:
            return 0.0, promised
        tokens = sum(int(s) for s in batch_seqlens)
        total = 6.0 * self._dense_params_per_token() * tokens + self._attention_flops(batch_seqlens)
        return total / delta_time / 1e12, promised
