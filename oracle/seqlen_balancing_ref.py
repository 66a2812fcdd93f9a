"""ORACLE — pure-Python restatement of the reference's Karmarkar-Karp partitioner (TEST
INFRASTRUCTURE: only tests/ may import this; the product path is va_karmarkar_karp).

Restates verl/utils/seqlen_balancing.py:26-127 with plain tuples instead of the reference's
classes, keeping every ordering rule that decides the result:
  * items are processed in ascending (value, index) order (:102);
  * a partition orders by (sum, item count, item tuple list) (:41-46);
  * a state keeps its partitions in descending order via a stable sort (:57, :70);
  * the state popped first has the largest spread, ties broken by the larger first partition
    (:76-82); two states popped in sequence merge partition i with partition k-1-i of the
    second (:67-70).
Pinned by the reference's own tests (tests/utils/test_seqlen_balancing.py: permutation round
trips, micro-batch counts under min_num_micro_batch / same_micro_num_in_dp) and by hand-checked
small cases in tests/test_seqlen_balancing.py.
"""

from __future__ import annotations


def _key(part):
    total, items = part
    return (total, len(items), items)


def _desc(parts):
    return sorted(parts, key=_key, reverse=True)


def _pop_key(state):
    return (state[0][0] - state[-1][0], _key(state[0]))


def karmarkar_karp(seqlens, k, equal_size):
    ranked = sorted((v, i) for i, v in enumerate(seqlens))
    empty = (0, ())

    def make(chunk):
        return _desc([(v, ((i, v),)) for v, i in chunk] + [empty] * (k - len(chunk)))

    if equal_size:
        assert len(ranked) % k == 0
        states = [make(ranked[o : o + k]) for o in range(0, len(ranked), k)]
    else:
        states = [make([r]) for r in ranked]
    while len(states) > 1:
        a = max(range(len(states)), key=lambda j: _pop_key(states[j]))
        first = states.pop(a)
        b = max(range(len(states)), key=lambda j: _pop_key(states[j]))
        second = states.pop(b)
        merged = [(x[0] + y[0], x[1] + y[1]) for x, y in zip(first, reversed(second))]
        states.append(_desc(merged))
    return [[i for i, _ in part[1]] for part in states[0]]
