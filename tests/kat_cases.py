"""Known answers derived by hand from the reference source (no oracle, no reference run): each case
states the inputs, the expected outputs worked out from the cited lines, and the working. Used twice:
tests/test_oracle_kats.py pins the CPU oracle to them, tests/test_kats_gpu.py pins the HIP kernels
to them directly, so neither side rests only on the other.
"""

import math

E = math.e

# ---- dual-clip PPO, core_algos.py:722-794 (cliprange 0.2, clip_ratio_c 3.0, one token per case) ----
# ratio = exp(clamp(lp - old, -20, 20)); l1 = -A r; l2 = -A clamp(r, 0.8, 1.2); lmax = max(l1, l2)
# A >= 0: per-token lmax; A < 0: min(lmax, -A c). clipfrac counts l2 > l1, clipfrac_lower counts
# lmax > -A c with A < 0.
#   (A, lp - old)   r        l1        l2     per-token   clip  lower
#   (+1, 0.5)      e^0.5    -1.6487   -1.2    -1.2        1     0     (upper clip, A > 0)
#   (-1, 1.5)      e^1.5    +4.4817   +1.2    +3.0        0     1     (dual clip: min(4.4817, 3))
#   (-1, -0.5)     e^-0.5   +0.6065   +0.8    +0.8        1     0     (lower clip, A < 0)
#   (+2, 0)        1        -2        -2      -2          0     0     (inside the trust region)
# Every mean is masked_mean = masked sum / (mask count + 1e-8) (torch_functional.py:171-185).
_N4 = 4 + 1e-8
POLICY_CASE = dict(
    adv=[1.0, -1.0, -1.0, 2.0],
    d_lp=[0.5, 1.5, -0.5, 0.0],
    per_token=[-1.2, 3.0, 0.8, -2.0],
    pg_loss=(-1.2 + 3.0 + 0.8 - 2.0) / _N4,  # token-mean: 0.15
    clipfrac=2 / _N4,
    clipfrac_lower=1 / _N4,
    ppo_kl=-(0.5 + 1.5 - 0.5 + 0.0) / _N4,  # masked_mean(-(lp - old)): -0.375
    # d pg_loss / d lp (token-mean over 4): only the unclipped branches carry the ratio's gradient:
    # case 1 clipped (0), case 2 the constant dual bound (0), case 3 clipped (0), case 4 -A r / 4
    # (at r = 1 l1 == l2: torch.maximum splits the gradient, both halves -A r)
    dlp=[0.0, 0.0, 0.0, -2.0 * 1.0 / _N4],
)

# lp - old is clamped to [-20, 20] before exp AND before the KL metric (core_algos.py:766-770):
# lp - old = 25 with A = -1 gives r = e^20, l1 = e^20 > 3, so the dual clip yields 3, clipfrac_lower 1,
# and ppo_kl = masked_mean(-clamped) = -20, not -25
_N1 = 1 + 1e-8
CLAMP_CASE = dict(adv=[-1.0], d_lp=[25.0], pg_loss=3.0 / _N1, clipfrac=0.0, clipfrac_lower=1.0 / _N1,
                  ppo_kl=-20.0 / _N1)

# ---- agg_loss, core_algos.py:686-719 ----
AGG_LOSS = [[1.0, 2.0, 3.0], [4.0, 5.0, 6.0]]
AGG_MASK = [[1, 1, 0], [1, 0, 0]]
AGG_WANT = {
    "token-mean": (1 + 2 + 4) / (3 + 1e-8),  # masked_mean
    "seq-mean-token-sum": (3 + 4) / 2,  # mean over rows of the row sums
    "seq-mean-token-mean": (3 / 2 + 4 / 1) / 2,  # mean over rows of the row means
    "seq-mean-token-sum-norm": (3 + 4) / 3,  # total / the mask's last dim (3)
}

# ---- kl_penalty, core_algos.py:1034-1069 (logprob, ref_logprob) -> value ----
#   k1 = lp - ref; abs = |lp - ref|; k2 = (lp - ref)^2 / 2; k3: k = clamp(ref - lp, -20, 20),
#   clamp(e^k - k - 1, -10, 10)
KL_LP = [0.0, -1.0, 0.0, -30.0]
KL_REF = [-1.0, 0.0, 0.0, 0.0]
KL_WANT = {
    "kl": [1.0, -1.0, 0.0, -30.0],
    "abs": [1.0, 1.0, 0.0, 30.0],
    "mse": [0.5, 0.5, 0.0, 450.0],
    "low_var_kl": [1 / E, E - 2.0, 0.0, 10.0],  # k = -1: e^-1; k = 1: e - 2; k = 20 (clamped): 10
}

# ---- masked_whiten, torch_functional.py:206-223: unbiased variance, rsqrt(var + 1e-8) ----
WHITEN_X = [1.0, 2.0, 3.0, 4.0, 100.0]
WHITEN_MASK = [1, 1, 1, 1, 0]
# mean 2.5; unbiased var = (2.25 + 0.25 + 0.25 + 2.25) / 3 = 5 / 3
# (masked_mean's 1e-8: mean = 10 / (4 + 1e-8); masked_var's own bias correction n / (n - 1))
_MU = 10 / (4 + 1e-8)
_VAR = sum((x - _MU) ** 2 for x in WHITEN_X[:4]) / (4 + 1e-8) * 4 / 3
WHITEN_WANT = [(x - _MU) / math.sqrt(_VAR + 1e-8) for x in WHITEN_X]

# ---- GRPO outcome advantage, core_algos.py:246-308 (epsilon 1e-6) ----
# group "a": scores 1, 0, 0, 1 -> mean 0.5, unbiased std sqrt(1/3); group "b": singleton -> (0, 1)
GRPO_SCORES = [1.0, 0.0, 0.0, 1.0, 5.0]
GRPO_UID = ["a", "a", "a", "a", "b"]
_S = math.sqrt(1 / 3)
GRPO_WANT = [0.5 / (_S + 1e-6), -0.5 / (_S + 1e-6), -0.5 / (_S + 1e-6), 0.5 / (_S + 1e-6), 5.0 / (1.0 + 1e-6)]
GRPO_NOSTD_WANT = [0.5, -0.5, -0.5, 0.5, 5.0]  # Dr.GRPO: scores - mean (singleton mean 0)

# ---- log-softmax gather + entropy in closed form (torch_functional.py:64-160; dp_actor.py:182-201) ----
# Row r has k_r logits at the value c_r and V - k_r at 0 (the "hot" entries are the first k_r), so
#   Z = k e^c + (V - k), lse = ln Z, logp(label) = c [label < k] - lse,
#   H = lse - sum p x = ln Z - k c e^c / Z,
# and the gradients d logp / d x_j = [j = label] - p_j, d H / d x_j = -p_j (x_j - lse + H)
# (p_j = e^{x_j} / Z); with a temperature T the logits are x / T and the gradients gain a 1 / T.
LS_V = 1000
LS_ROWS = [  # (k, c, label): c and c / 2 are exact in bf16
    (0, 0.0, 7),  # uniform: logp = -ln V, H = ln V
    (1, 2.0, 0),  # one hot entry, label on it
    (10, 3.0, 500),  # label on a cold entry
    (500, -1.0, 3),  # half the row below zero, label hot
    (999, 4.0, 999),  # all but the last entry hot, label the cold tail entry
]


def ls_logits(temperature=1.0):
    """[rows, V] logits (before the division by T) and labels of LS_ROWS, as nested lists."""
    rows = [[c if j < k else 0.0 for j in range(LS_V)] for k, c, _ in LS_ROWS]
    return rows, [lab for _, _, lab in LS_ROWS]


def ls_expected(temperature=1.0, g_logp=1.0, g_ent=0.5):
    """(logp, entropy, dlogits) of LS_ROWS in closed form (floats; dlogits the gradient of
    g_logp * logp + g_ent * H with respect to the UNDIVIDED logits)."""
    logp, ent, grads = [], [], []
    for k, c, lab in LS_ROWS:
        z = c / temperature
        Z = k * math.exp(z) + (LS_V - k)
        lse = math.log(Z)
        H = lse - k * z * math.exp(z) / Z
        logp.append((z if lab < k else 0.0) - lse)
        ent.append(H)
        g = []
        for j in range(LS_V):
            x = z if j < k else 0.0
            p = math.exp(x) / Z
            g.append((g_logp * ((1.0 if j == lab else 0.0) - p) + g_ent * (-p * (x - lse + H))) / temperature)
        grads.append(g)
    return logp, ent, grads


# ---- outcome estimators (core_algos.py:311-605), worked by hand ----
def _masked_whiten(vals, mask):
    """torch_functional.py:171-223 on flat lists: masked_mean with its + 1e-8, unbiased variance
    (masked_mean of the squared deviations times n / (n - 1)), rsqrt(var + 1e-8)."""
    n = sum(mask)
    mu = sum(v * m for v, m in zip(vals, mask)) / (n + 1e-8)
    var = sum((v - mu) ** 2 * m for v, m in zip(vals, mask)) / (n + 1e-8) * n / (n - 1)
    return [(v - mu) / math.sqrt(var + 1e-8) for v in vals]


# RLOO (core_algos.py:428-476): a_i = (s_i - mean) n / (n - 1) within a group; a singleton keeps s
RLOO_SCORES, RLOO_UID = [1.0, 0.0, 0.0, 1.0, 5.0], ["a", "a", "a", "a", "b"]
RLOO_WANT = [2 / 3, -2 / 3, -2 / 3, 2 / 3, 5.0]

# OPO (core_algos.py:479-530): baseline sum(len s) / sum(len) per group (singleton: 0), len = mask sum
OPO_SCORES, OPO_UID, OPO_LEN = [1.0, 0.0, 1.0, 7.0], ["a", "a", "a", "b"], [2, 1, 1, 3]
OPO_WANT = [0.25, -0.75, 0.25, 7.0]  # group a: (2 * 1 + 1 * 0 + 1 * 1) / 4 = 0.75

# pass@k (core_algos.py:311-370): only the group's best gets (r_max - r_2nd) / (std + eps)
PASSK_SCORES, PASSK_UID = [1.0, 3.0, 2.0], ["a", "a", "a"]
PASSK_WANT = [0.0, 1.0 / (1.0 + 1e-6), 0.0]  # unbiased std of (1, 3, 2) = 1
PASSK_NOSTD_WANT = [0.0, 1.0, 0.0]

# REINFORCE++ (core_algos.py:533-569), gamma 0.5: running = r_t + gamma running, stored, then reset
# by the mask. Row 0 [0, 0, 1] all valid -> [0.25, 0.5, 1]; row 1 [1, 0, 2] with mask [1, 1, 0] ->
# t = 2: 2 (stored, then reset to 0), t = 1: 0, t = 0: 1 -> [1, 0, 2]; advantages = masked_whiten of
# the returns over the 5 valid entries, times the mask
RFPP_REWARDS = [[0.0, 0.0, 1.0], [1.0, 0.0, 2.0]]
RFPP_MASK = [[1, 1, 1], [1, 1, 0]]
RFPP_RETURNS = [[0.25, 0.5, 1.0], [1.0, 0.0, 2.0]]
_w = _masked_whiten([0.25, 0.5, 1.0, 1.0, 0.0, 2.0], [1, 1, 1, 1, 1, 0])
RFPP_ADV = [_w[:3], [_w[3], _w[4], 0.0]]

# ReMax (core_algos.py:572-605): returns = reverse cumsum of r * mask; adv = returns - b * mask
REMAX_REWARDS, REMAX_MASK, REMAX_BASE = [[0.0, 0.0, 1.0, 5.0]], [[1, 1, 1, 0]], [0.25]
REMAX_RETURNS = [[1.0, 1.0, 1.0, 0.0]]
REMAX_ADV = [[0.75, 0.75, 0.75, 0.0]]

# GAE (core_algos.py:193-241), gamma = lam = 0.5, values [0.1, 0.2, 0.3], reward 1 at the end:
# delta_2 = 1 - 0.3 = 0.7, delta_1 = 0.5 * 0.3 - 0.2 = -0.05, delta_0 = 0.5 * 0.2 - 0.1 = 0
# A_2 = 0.7, A_1 = -0.05 + 0.25 * 0.7 = 0.125, A_0 = 0 + 0.25 * 0.125 = 0.03125; returns = A + V
GAE_REWARDS, GAE_VALUES, GAE_MASK = [[0.0, 0.0, 1.0]], [[0.1, 0.2, 0.3]], [[1, 1, 1]]
GAE_RETURNS = [[0.13125, 0.325, 1.0]]
GAE_ADV = [_masked_whiten([0.03125, 0.125, 0.7], [1, 1, 1])]


# ---- registered loss variants (core_algos.py:797-972), one row of 4 tokens, mask 1, token-mean ----
# gpg: -lp A aggregated; metrics 0. lp = [0.1, -0.2, 0.4, 0], A = [1, -1, 2, 0]:
#   losses [-0.1, -0.2, -0.8, 0] -> -1.1 / 4; d/dlp = -A / 4
GPG_LP, GPG_ADV = [0.1, -0.2, 0.4, 0.0], [1.0, -1.0, 2.0, 0.0]
GPG_LOSS = -1.1 / _N4
GPG_DLP = [-1.0 / _N4, 1.0 / _N4, -2.0 / _N4, 0.0]
# kl_cov (kl_cov_ratio 0.25 -> k = max(1, int(4 * 0.25)) = 1 token, ppo_kl_coef 1), old = 0: cov =
# (A - 0.5)(lp - 0.075) = [0.0125, 0.4125, 0.4875, 0.0375] -> token 2 gets + |lp - old| = 0.4:
#   losses [-e^0.1, e^-0.2, -2 e^0.4 + 0.4, 0]; ppo_kl (slot 2) = masked_mean |lp - old| = 0.7 / 4;
#   d/dlp = [-e^0.1, e^-0.2, -2 e^0.4 + 1, 0] / 4
KLCOV_LOSS = (-math.exp(0.1) + math.exp(-0.2) - 2 * math.exp(0.4) + 0.4) / _N4
KLCOV_PPO_KL = 0.7 / _N4
KLCOV_DLP = [-math.exp(0.1) / _N4, math.exp(-0.2) / _N4, (-2 * math.exp(0.4) + 1.0) / _N4, 0.0]
# clip_cov (clip_cov_ratio 0.25 -> 1 token, bounds (1, 5)), lp = old = [1, -0.3, -0.7, 0] (ratio 1,
# nothing clipped by the ratio), A = [2, -2, 0, 0]: cov = A (lp - 0) = [2, 0.6, 0, 0], only token 0 lies
# in (1, 5), so the random draw has one candidate: corr = [0, 1, 1, 1];
#   losses max(l1, l2) corr = [0, 2, 0, 0] -> 2 / 4; clipfrac = 1 / 4; ppo_kl 0;
#   d/dlp: token 1 at the l1 == l2 tie, torch.maximum's halves both -A r = 2 -> 2 / 4
CLIPCOV_LP, CLIPCOV_ADV = [1.0, -0.3, -0.7, 0.0], [2.0, -2.0, 0.0, 0.0]
CLIPCOV_LOSS = 2.0 / _N4
CLIPCOV_CLIPFRAC = 1.0 / _N4
CLIPCOV_DLP = [0.0, 2.0 / _N4, 0.0, 0.0]
