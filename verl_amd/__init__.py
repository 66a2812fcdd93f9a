"""verl_amd — MI355X-native PPO/GRPO actor-update hot path for verl.

Drop-in mirror of the reference's hot-path API (rfahrn/verl 0.4.1.dev):
  verl_amd.protocol.DataProto                 <- verl/protocol.py
  verl_amd.utils.torch_functional             <- verl/utils/torch_functional.py
  verl_amd.trainer.ppo.core_algos             <- verl/trainer/ppo/core_algos.py
  verl_amd.trainer.ppo.ray_trainer            <- compute_advantage / apply_kl_penalty
  verl_amd.workers.actor.DataParallelPPOActor <- verl/workers/actor/dp_actor.py
The arithmetic runs in hand-written gfx950 HIP kernels (verl_amd/csrc, C-ABI in
include/verl_amd.h) loaded from verl_amd/lib/libverl_amd.so.
"""

__version__ = "0.1.0"
