"""Model builders for the actor-update benchmark and tests.

No checkpoints or network exist on the boxes, so models are HF architectures instantiated from
locally written configs with random init. Qwen2.5-0.5B: hidden 896 and vocab 151,936 are
confirmed by the reference (tests/utils/test_linear_cross_entropy.py:121-125); the remaining
values (24 layers, 14 query heads, 2 KV heads, FFN 4864, tied embeddings, rope theta 1e6) are
the public model card's and are recorded as assumptions in DESIGN.md.
"""

from __future__ import annotations

import torch


def qwen2_config(size: str = "0.5b", **overrides):
    from transformers import Qwen2Config

    presets = {
        "0.5b": dict(hidden_size=896, intermediate_size=4864, num_hidden_layers=24, num_attention_heads=14,
                     num_key_value_heads=2, vocab_size=151936, tie_word_embeddings=True),
        # BASELINE config 5 (DAPO): the public Qwen2.5-7B card's values (assumed, no checkpoint here)
        "7b": dict(hidden_size=3584, intermediate_size=18944, num_hidden_layers=28, num_attention_heads=28,
                   num_key_value_heads=4, vocab_size=152064, tie_word_embeddings=False),
        "tiny": dict(hidden_size=128, intermediate_size=352, num_hidden_layers=2, num_attention_heads=4,
                     num_key_value_heads=2, vocab_size=4096, tie_word_embeddings=True),
    }
    kw = dict(presets[size])
    kw.update(max_position_embeddings=32768, rope_theta=1000000.0, rms_norm_eps=1e-6, use_sliding_window=False,
              hidden_act="silu", attention_dropout=0.0, torch_dtype="float32")
    kw.update(overrides)
    return Qwen2Config(**kw)


def build_qwen2(size: str = "0.5b", device="cuda", dtype=torch.float32, seed: int = 0, **overrides):
    from transformers import Qwen2ForCausalLM

    torch.manual_seed(seed)
    cfg = qwen2_config(size, **overrides)
    with torch.device(device):
        model = Qwen2ForCausalLM(cfg)
    return model.to(dtype)


def create_random_mask(input_ids: torch.Tensor, max_ratio_of_valid_token: float, max_ratio_of_left_padding: float,
                       min_ratio_of_valid_token: float = 0):
    """verl/utils/model.py:176-216 — a random left-padded / right-padded 0/1 mask (numpy RNG)."""
    import numpy as np

    assert 0 < max_ratio_of_valid_token <= 1.0
    assert 0 <= max_ratio_of_left_padding < 1.0
    assert min_ratio_of_valid_token <= max_ratio_of_valid_token
    bs, seq = input_ids.shape
    max_valid = int(seq * max_ratio_of_valid_token)
    min_valid = max(1, int(seq * min_ratio_of_valid_token))
    max_left = int(seq * max_ratio_of_left_padding)
    assert max_valid + max_left <= seq
    masks = torch.ones_like(input_ids, dtype=torch.int64)
    for i in range(bs):
        left = int(np.random.randint(low=0, high=max_left + 1, dtype=np.int64))
        valid = int(np.random.randint(low=min_valid, high=max_valid + 1, dtype=np.int64))
        masks[i, :left] = 0
        masks[i, left + valid :] = 0
    return masks


def llama_config(size: str = "tiny", **overrides):
    """Llama-architecture configs (BASELINE config 3 is Llama-3-8B PPO with a critic). "8b" follows
    the public Llama-3-8B card (assumed: no checkpoint or network here); "tiny" keeps head_dim 64
    and Llama-3.1's rope scaling so the packed backbone's kernels and the scaled-RoPE path are
    exercised."""
    from transformers import LlamaConfig

    llama3_rope = dict(rope_type="llama3", factor=8.0, low_freq_factor=1.0, high_freq_factor=4.0,
                       original_max_position_embeddings=8192)
    presets = {
        "8b": dict(hidden_size=4096, intermediate_size=14336, num_hidden_layers=32, num_attention_heads=32,
                   num_key_value_heads=8, vocab_size=128256, tie_word_embeddings=False,
                   max_position_embeddings=8192, rope_scaling=None),
        "tiny": dict(hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4,
                     num_key_value_heads=2, vocab_size=4096, tie_word_embeddings=False,
                     max_position_embeddings=131072, rope_scaling=llama3_rope),
    }
    kw = dict(presets[size])
    kw.update(rope_theta=500000.0, rms_norm_eps=1e-5, hidden_act="silu", attention_dropout=0.0, attention_bias=False,
              mlp_bias=False, torch_dtype="float32")
    kw.update(overrides)
    return LlamaConfig(**kw)


def build_llama(size: str = "tiny", device="cuda", dtype=torch.float32, seed: int = 0, **overrides):
    from transformers import LlamaForCausalLM

    torch.manual_seed(seed)
    cfg = llama_config(size, **overrides)
    with torch.device(device):
        model = LlamaForCausalLM(cfg)
    return model.to(dtype)


def build_llama_critic(size: str = "tiny", device="cuda", dtype=torch.float32, seed: int = 0, **overrides):
    """Llama value model as the reference builds its critic (fsdp_workers.py:1018-1031)."""
    from transformers import LlamaForTokenClassification

    torch.manual_seed(seed)
    cfg = llama_config(size, **overrides)
    cfg.num_labels = 1
    cfg.classifier_dropout = 0.0
    with torch.device(device):
        model = LlamaForTokenClassification(cfg)
    return model.to(dtype)


def build_qwen2_critic(size: str = "0.5b", device="cuda", dtype=torch.float32, seed: int = 0, **overrides):
    """The reference's critic: AutoModelForTokenClassification with num_labels = 1 and
    classifier_dropout = 0 (fsdp_workers.py:1018-1031) on the Qwen2 architecture, random init."""
    from transformers import Qwen2ForTokenClassification

    torch.manual_seed(seed)
    cfg = qwen2_config(size, **overrides)
    cfg.num_labels = 1
    cfg.classifier_dropout = 0.0
    with torch.device(device):
        model = Qwen2ForTokenClassification(cfg)
    return model.to(dtype)


def qwen2_vl_config(size: str = "tiny", **text_overrides):
    """Qwen2-VL configs (BASELINE config 4: Qwen2-VL-7B GRPO). "7b" follows the public
    Qwen2-VL-7B-Instruct card (assumed: no checkpoint or network here): Qwen2 decoder with
    multimodal RoPE sections (16, 24, 24) over head_dim 128, and a 32-block ViT (embed 1280, 16
    heads, 14-px patches, 2 x 2 spatial merge). "tiny" keeps head_dim 64 so the gfx950 flash
    kernels run, with sections (8, 12, 12)."""
    from transformers import Qwen2VLConfig

    presets = {
        "7b": (dict(hidden_size=3584, intermediate_size=18944, num_hidden_layers=28, num_attention_heads=28,
                    num_key_value_heads=4, vocab_size=152064, tie_word_embeddings=False, mrope_section=[16, 24, 24]),
               dict(depth=32, embed_dim=1280, hidden_size=3584, num_heads=16, mlp_ratio=4),
               dict(image_token_id=151655, video_token_id=151656, vision_start_token_id=151652,
                    vision_end_token_id=151653, bos_token_id=151643, eos_token_id=151645)),
        "tiny": (dict(hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4,
                      num_key_value_heads=2, vocab_size=4096, tie_word_embeddings=False, mrope_section=[8, 12, 12]),
                 dict(depth=1, embed_dim=64, hidden_size=256, num_heads=4, mlp_ratio=2),
                 dict(image_token_id=4091, video_token_id=4092, vision_start_token_id=4093, vision_end_token_id=4094,
                      bos_token_id=4090, eos_token_id=4095)),
    }
    text, vision, tokens = (dict(d) for d in presets[size])
    sec = text.pop("mrope_section")
    text.update(rope_theta=1000000.0, rms_norm_eps=1e-6, max_position_embeddings=32768, use_sliding_window=False,
                hidden_act="silu", attention_dropout=0.0, rope_scaling={"type": "mrope", "mrope_section": sec})
    text.update(text_overrides)
    vision.update(patch_size=14, spatial_merge_size=2, temporal_patch_size=2, in_channels=3)
    tie = text.pop("tie_word_embeddings")
    return Qwen2VLConfig(text_config=dict(text, tie_word_embeddings=tie, bos_token_id=tokens["bos_token_id"],
                                          eos_token_id=tokens["eos_token_id"]),
                         vision_config=vision, tie_word_embeddings=tie, **tokens)


def build_qwen2_vl(size: str = "tiny", device="cuda", dtype=torch.float32, seed: int = 0, **text_overrides):
    from transformers import Qwen2VLForConditionalGeneration

    torch.manual_seed(seed)
    cfg = qwen2_vl_config(size, **text_overrides)
    with torch.device(device):
        model = Qwen2VLForConditionalGeneration(cfg)
    return model.to(dtype)
