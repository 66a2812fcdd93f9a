"""Per-GPU actor worker — the update_actor / compute_log_prob surface of
verl/workers/fsdp_workers.py:105-916 (ActorRolloutRefWorker) without Ray or FSDP.

One process per GPU (launched by torch.distributed.run or by the caller), torch.distributed
over RCCL for device tensors. Every rank holds full fp32 parameters; gradients are averaged
with the bucketed all-reduce of grad_sync.py. The DP_COMPUTE_PROTO contract of the reference
(decorator.py:375-408: chunk the batch by DP rank, run, concat) is available as
dispatch_dp_compute_data_proto / collect_dp_compute_data_proto for a caller holding the full
batch; an SPMD caller passes each rank its own shard directly.
"""

from __future__ import annotations

import os
import time

import torch
import torch.distributed as dist

from ..protocol import DataProto
from ..utils.flops_counter import FlopsCounter
from ..utils.torch_functional import build_lr_scheduler
from .actor import DataParallelPPOActor
from .actor.dp_actor import DeviceMetrics
from .grad_sync import FlatAdamW, GradBucketReducer, MixedPrecisionParams, ShardedMixedPrecisionParams


def init_distributed(backend: str | None = None) -> tuple[int, int]:
    """fsdp_workers.py:118-126: init the process group from the torchrun env (127.0.0.1).

    ``VA_DIST_BACKEND`` overrides the backend (``gloo`` lets several ranks share one GPU for a
    rehearsal of the multi-rank path; RCCL needs one GPU per rank)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = os.environ.get("VA_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        local = local_device_index()
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                device_id=torch.device("cuda", local) if backend == "nccl" else None)
    return rank, world


def local_device_index() -> int:
    """LOCAL_RANK folded onto the visible GPUs (more ranks than GPUs only under VA_DIST_BACKEND=gloo)."""
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n = torch.cuda.device_count()  # counts devices without initialising HIP
    return local % n if n > 0 else local


def dispatch_dp_compute_data_proto(data: DataProto, world_size: int) -> list[DataProto]:
    """decorator.py:375-385: equal chunks, one per DP rank."""
    return data.chunk(chunks=world_size)


def collect_dp_compute_data_proto(outputs: list[DataProto]) -> DataProto:
    """decorator.py:399-408."""
    return DataProto.concat(outputs)


def make_param_manager(module: torch.nn.Module, bucket_mb: int, mixed_precision: bool, zero: bool):
    """Parameter / gradient / optimizer-state layout of a trained role (see grad_sync.py)."""
    if zero:
        if not mixed_precision:
            raise ValueError("zero=True shards the fp32 masters of the bf16 mixed-precision layout")
        return ShardedMixedPrecisionParams(module, bucket_bytes=bucket_mb << 20)
    if mixed_precision:
        return MixedPrecisionParams(module, bucket_bytes=bucket_mb << 20)
    return GradBucketReducer(module.parameters(), bucket_bytes=bucket_mb << 20)


# VERL_AMD_FLAT_ADAMW=0: torch.optim.AdamW(fused=True) over the masters instead of grad_sync.FlatAdamW
_FLAT_ADAMW = os.environ.get("VERL_AMD_FLAT_ADAMW", "1") != "0"


def make_optimizer(manager, optim, fused: bool):
    """AdamW with the role's optim config (fsdp_workers.py:418-423): FlatAdamW over the replicated
    mixed-precision manager's flat buckets on the GPU, torch's AdamW otherwise (fused on the GPU)."""
    betas = tuple(optim.get("betas", (0.9, 0.999)))
    wd = optim.get("weight_decay", 0.01)
    if fused and _FLAT_ADAMW and isinstance(manager, MixedPrecisionParams):
        return FlatAdamW(manager, lr=optim.lr, betas=betas, weight_decay=wd)
    return torch.optim.AdamW(manager.optimizer_params(), lr=optim.lr, betas=betas, weight_decay=wd, fused=fused)


class ActorWorker:
    """update_actor / compute_log_prob of the actor role, one per GPU."""

    def __init__(self, config, rollout_n: int = 1):
        self.config = config
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.world_size = dist.get_world_size() if dist.is_initialized() else 1
        actor = config.actor
        # batch-size normalisation, fsdp_workers.py:174-196 (sp = 1)
        actor.ppo_mini_batch_size = actor.ppo_mini_batch_size * rollout_n // self.world_size
        assert actor.ppo_mini_batch_size > 0, "ppo_mini_batch_size must be > 0 after normalisation"
        if actor.get("ppo_micro_batch_size_per_gpu") is None and actor.get("ppo_micro_batch_size") is not None:
            actor.ppo_micro_batch_size_per_gpu = actor.ppo_micro_batch_size // self.world_size
        if actor.get("ppo_micro_batch_size_per_gpu") is not None:
            assert actor.ppo_mini_batch_size % actor.ppo_micro_batch_size_per_gpu == 0, (
                f"normalized ppo_mini_batch_size {actor.ppo_mini_batch_size} should be divisible by "
                f"ppo_micro_batch_size_per_gpu {actor.ppo_micro_batch_size_per_gpu}"
            )
        elif not actor.get("use_dynamic_bsz", False):
            raise ValueError("ppo_micro_batch_size_per_gpu is required unless use_dynamic_bsz is set")
        self.actor = None
        self.module = None
        self.ref_policy = None

    def init_model(self, module: torch.nn.Module, bucket_mb: int = 256, mixed_precision: bool = True,
                   zero: bool = False):
        """fsdp_workers.py:562-670 (model already built by the caller; AdamW with the actor's optim
        config, fsdp_workers.py:418-423). mixed_precision=True is the FSDP MixedPrecision of the
        reference (bf16 compute weights, fp32 master weights / grads / reduction, :337-347).
        zero=True shards the fp32 masters and AdamW state over the ranks (FSDP FULL_SHARD's
        optimizer-state saving, :94-99, 371; grad_sync.ShardedMixedPrecisionParams)."""
        self.module = module
        optim = self.config.actor.optim
        fused = next(module.parameters()).is_cuda
        manager = make_param_manager(module, bucket_mb, mixed_precision, zero)
        opt = make_optimizer(manager, optim, fused)
        self.actor = DataParallelPPOActor(self.config.actor, module, opt, grad_reducer=manager)
        self.actor_optimizer = opt
        self.actor_lr_scheduler = build_lr_scheduler(opt, optim, role="actor", rank=self.rank)
        self.flops_counter = FlopsCounter(module.config)
        return self

    def init_ref_model(self, module: torch.nn.Module, mixed_precision: bool = True):
        """The reference policy held next to the actor (fsdp_workers.py:578-591, `_is_ref`): a frozen
        copy run by a DataParallelPPOActor without optimizer (dp_actor.py:52-53), in bf16 like the
        reference's FSDP param_dtype when mixed_precision."""
        if mixed_precision:
            for p in module.parameters():
                p.data = p.data.to(torch.bfloat16)
        for p in module.parameters():
            p.requires_grad_(False)
        self.ref_policy = DataParallelPPOActor(self.config.actor, module, None)
        return self

    def compute_ref_log_prob(self, data: DataProto) -> DataProto:
        """fsdp_workers.py:802-835: ref_log_prob for this rank's shard (no entropy)."""
        ref = self.config.get("ref") or {}
        ro = self.config.rollout
        data.meta_info["micro_batch_size"] = ref.get("log_prob_micro_batch_size_per_gpu",
                                                     ro.get("log_prob_micro_batch_size_per_gpu"))
        data.meta_info["temperature"] = ro.temperature
        data.meta_info["max_token_len"] = ref.get("log_prob_max_token_len_per_gpu",
                                                  ro.get("log_prob_max_token_len_per_gpu", 16384))
        data.meta_info["use_dynamic_bsz"] = ref.get("log_prob_use_dynamic_bsz", ro.get("log_prob_use_dynamic_bsz", False))
        lp, _ = self.ref_policy.compute_log_prob(data, calculate_entropy=False)
        return DataProto.from_dict(tensors={"ref_log_prob": lp})

    def compute_log_prob(self, data: DataProto) -> DataProto:
        """fsdp_workers.py:758-800: old_log_probs (+ entropys) for this rank's shard."""
        ro = self.config.rollout
        data.meta_info.setdefault("micro_batch_size", ro.get("log_prob_micro_batch_size_per_gpu"))
        data.meta_info.setdefault("temperature", ro.temperature)
        data.meta_info.setdefault("use_dynamic_bsz", ro.get("log_prob_use_dynamic_bsz", False))
        data.meta_info.setdefault("max_token_len", ro.get("log_prob_max_token_len_per_gpu", 16384))
        lp, ent = self.actor.compute_log_prob(data, calculate_entropy=True)
        return DataProto.from_dict(tensors={"old_log_probs": lp, "entropys": ent},
                                   meta_info={"temperature": data.meta_info["temperature"]})

    def compute_advantage(self, data: DataProto, adv_estimator, gamma: float = 1.0, lam: float = 1.0,
                          num_repeat: int = 1, norm_adv_by_std_in_grpo: bool = True, config=None) -> DataProto:
        """The driver's compute_advantage (ray_trainer.py:214-291, called at :1297) run here on
        this rank's shard, on the GPU: batch-global statistics (GRPO-family group stats, GAE /
        RF++ whitening) are exchanged over the process group (trainer/ppo/dp_algos.py), so the
        result equals the reference's whole-batch computation whether or not prompt groups were
        split over ranks by _balance_batch."""
        from ..trainer.ppo.dp_algos import compute_advantage_dp

        return compute_advantage_dp(data, adv_estimator, gamma=gamma, lam=lam, num_repeat=num_repeat,
                                    norm_adv_by_std_in_grpo=norm_adv_by_std_in_grpo, config=config)

    def update_actor(self, data: DataProto) -> DataProto:
        """fsdp_workers.py:672-716: one PPO update; metrics in meta_info, with the RPC's own
        additions: perf/mfu/actor (model FLOPs of the whole batch's tokens, meta_info
        global_token_num, over the update's wall time and the device peak, / world size),
        perf/max_memory_* and perf/cpu_memory_used_gb, actor/lr (the rate this update used),
        then one LR-scheduler step. update_policy's metrics arrive by an asynchronous device->host
        copy (dp_actor.DeviceMetrics: the host does not wait for the update here), so the update's
        time for the MFU is its device span between two stream events, read with the metrics."""
        span = _UpdateSpan(self.module)
        metrics = as_device_metrics(self.actor.update_policy(data))
        span.stop()
        epochs = self.config.actor.get("ppo_epochs", 1)
        metrics.update(perf_metrics(self.flops_counter, data, span.host_seconds(), epochs, self.world_size, "actor"))
        # the callback holds the token counts only, not the batch
        tokens, share = token_share(data, self.world_size)
        fc = self.flops_counter
        metrics.add_on_ready(lambda m: m.__setitem__("perf/mfu/actor", mfu(fc, tokens, share, span.seconds(), epochs)))
        metrics["actor/lr"] = self.actor_lr_scheduler.get_last_lr()[0]
        self.actor_lr_scheduler.step()
        return DataProto(meta_info={"metrics": metrics})


class CriticWorker:
    """compute_values / update_critic of the critic role, one per GPU (fsdp_workers.py:931-1265
    without FSDP / Ulysses / offload: plain DP over RCCL with bf16 compute + fp32 masters)."""

    def __init__(self, config):
        self.config = config
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.world_size = dist.get_world_size() if dist.is_initialized() else 1
        c = config
        # normalisation, fsdp_workers.py:953-975 (sp = 1)
        c.ppo_mini_batch_size = c.ppo_mini_batch_size * c.get("rollout_n", 1) // self.world_size
        if c.get("ppo_micro_batch_size") is not None:
            c.ppo_micro_batch_size //= self.world_size
            c.forward_micro_batch_size //= self.world_size
            c.ppo_micro_batch_size_per_gpu = c.ppo_micro_batch_size
            c.forward_micro_batch_size_per_gpu = c.forward_micro_batch_size
        if c.get("ppo_micro_batch_size_per_gpu") is not None:
            assert c.ppo_mini_batch_size % c.ppo_micro_batch_size_per_gpu == 0, (
                f"normalized ppo_mini_batch_size {c.ppo_mini_batch_size} should be divisible by "
                f"ppo_micro_batch_size_per_gpu {c.ppo_micro_batch_size_per_gpu}"
            )
            assert c.ppo_mini_batch_size // c.ppo_micro_batch_size_per_gpu > 0
        if c.get("forward_micro_batch_size_per_gpu") is None:
            c.forward_micro_batch_size_per_gpu = c.get("ppo_micro_batch_size_per_gpu")
        self.critic = None

    def init_model(self, module: torch.nn.Module, bucket_mb: int = 256, mixed_precision: bool = True,
                   zero: bool = False):
        from .critic import DataParallelPPOCritic

        optim = self.config.optim
        fused = next(module.parameters()).is_cuda
        manager = make_param_manager(module, bucket_mb, mixed_precision, zero)
        opt = make_optimizer(manager, optim, fused)
        self.critic = DataParallelPPOCritic(self.config, module, opt, grad_reducer=manager)
        self.critic_lr_scheduler = build_lr_scheduler(opt, optim, role="critic", rank=self.rank)
        self.flops_counter = FlopsCounter(module.config)
        return self

    def compute_values(self, data: DataProto) -> DataProto:
        """fsdp_workers.py:1207-1227."""
        data.meta_info["micro_batch_size"] = self.config.forward_micro_batch_size_per_gpu
        data.meta_info["max_token_len"] = self.config.forward_max_token_len_per_gpu
        data.meta_info["use_dynamic_bsz"] = self.config.use_dynamic_bsz
        values = self.critic.compute_values(data=data)
        return DataProto.from_dict(tensors={"values": values})

    def update_critic(self, data: DataProto) -> DataProto:
        """fsdp_workers.py:1231-1264: metrics + perf/mfu/critic + critic/lr, then one LR-scheduler
        step."""
        span = _UpdateSpan(getattr(self.critic, "critic_module", None))
        metrics = as_device_metrics(self.critic.update_critic(data=data))
        span.stop()
        epochs = self.config.get("ppo_epochs", 1)
        metrics["perf/mfu/critic"] = perf_metrics(self.flops_counter, data, span.host_seconds(), epochs,
                                                  self.world_size, "critic", memory=False)["perf/mfu/critic"]
        tokens, share = token_share(data, self.world_size)
        fc = self.flops_counter
        metrics.add_on_ready(lambda m: m.__setitem__("perf/mfu/critic", mfu(fc, tokens, share, span.seconds(), epochs)))
        metrics["critic/lr"] = self.critic_lr_scheduler.get_last_lr()[0]
        self.critic_lr_scheduler.step()
        return DataProto(meta_info={"metrics": metrics})


def as_device_metrics(metrics) -> DeviceMetrics:
    return metrics if isinstance(metrics, DeviceMetrics) else DeviceMetrics(metrics)


class _UpdateSpan:
    """Time of one update: its device span between two events on the current stream (the host
    does not wait for the update to finish), the host clock for a module off the GPU."""

    def __init__(self, module):
        p = next(module.parameters(), None) if module is not None else None
        self.cuda = p is not None and p.is_cuda
        self.t0 = time.perf_counter()
        self.t1 = None
        self.ev = None
        if self.cuda:
            self.ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            self.ev[0].record()

    def stop(self):
        self.t1 = time.perf_counter()
        if self.ev is not None:
            self.ev[1].record()

    def host_seconds(self) -> float:
        return self.t1 - self.t0

    def seconds(self) -> float:
        """The device span (waits for the end event), or the host time off the GPU."""
        if self.ev is None:
            return self.host_seconds()
        self.ev[1].synchronize()
        return self.ev[0].elapsed_time(self.ev[1]) / 1e3


def token_share(data: DataProto, world_size: int) -> tuple:
    """(per-sequence valid token counts, divisor) for the MFU: the whole batch's ``global_token_num``
    over the world size, or this rank's own attention mask undivided (see perf_metrics)."""
    tokens = data.meta_info.get("global_token_num")
    if tokens is None:
        return data.batch["attention_mask"].sum(-1).tolist(), 1
    return tokens, world_size


def mfu(flops_counter, tokens, share: int, delta_time: float, ppo_epochs: int) -> float:
    est, promised = flops_counter.estimate_flops(tokens, delta_time)
    return est * ppo_epochs / promised / share


def perf_metrics(flops_counter, data: DataProto, delta_time: float, ppo_epochs: int, world_size: int,
                 role: str, memory: bool = True) -> dict:
    """fsdp_workers.py:690-697: MFU of one update (estimated FLOP/s x epochs / promised / world)
    and the memory high-water marks. ``global_token_num`` lists the valid tokens of every sequence
    of the WHOLE batch (the reference's driver sets it before the DP dispatch, ray_trainer.py:1208;
    PPOTrainerStep and bench.py gather it over the ranks, metric_utils.global_token_num), so the
    whole batch's FLOPs are divided by the world size. Without it, this rank's own attention mask
    stands in, and then the FLOPs are already this rank's share: no division."""
    import psutil

    tokens, share = token_share(data, world_size)
    out = {f"perf/mfu/{role}": mfu(flops_counter, tokens, share, delta_time, ppo_epochs)}
    if not memory:
        return out
    if torch.cuda.is_available():
        out["perf/max_memory_allocated_gb"] = torch.cuda.max_memory_allocated() / (1024**3)
        out["perf/max_memory_reserved_gb"] = torch.cuda.max_memory_reserved() / (1024**3)
    out["perf/cpu_memory_used_gb"] = psutil.virtual_memory().used / (1024**3)
    return out
