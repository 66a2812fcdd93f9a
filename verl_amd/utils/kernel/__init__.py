"""Drop-ins for verl/utils/kernel/ (the reference's fused lm_head + log-prob + entropy kernels)."""
