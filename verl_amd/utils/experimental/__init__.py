"""Drop-ins for verl/utils/experimental/ (the reference's chunked-torch fused lm_head backend)."""
