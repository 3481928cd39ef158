"""Host model of the windowed symbol decoder's chain (decode.hip
dec_symw_kernel, BZ2MI_SYM_JUMP): the 64 lanes' successors (offset + code
length; 0 = a special code: longer than the lookup, or the end of block),
reachable-offset masks doubled until lane 0 leaves the window, the first
`budget` ordinary codes taken.  Checked against the sequential walk the
reference's decoder does (HuffmanStageDecoder::nextSymbol, one code after the
other) on random length vectors -- the rule the kernel's A/B fix pinned: a
budget that runs out right before a special code stops at the budget.
"""
from __future__ import annotations

import random


def sequential(lens, budget):
    o, taken = 0, []
    while True:
        if lens[o] == 0:
            return taken, o, True
        taken.append(o)
        o += lens[o]
        if len(taken) == budget or o >= 64:
            return taken, o, False


def jumping(lens, budget):
    J = [64 if lens[j] == 0 else min(j + lens[j], 64) for j in range(64)]
    R = [1 << j for j in range(64)]
    for _ in range(6):
        if J[0] >= 64:
            break
        R = [R[j] | (R[J[j]] if J[j] < 64 else 0) for j in range(64)]
        J = [J[J[j]] if J[j] < 64 else 64 for j in range(64)]
    orbit = R[0]
    special = sum(1 << j for j in range(64) if lens[j] == 0)
    ordinary = orbit & ~special
    taken = [j for j in range(64) if (ordinary >> j) & 1 and bin(ordinary & ((1 << j) - 1)).count("1") < budget]
    if len(taken) == budget:
        return taken, taken[-1] + lens[taken[-1]], False
    if orbit & special:
        return taken, (orbit & special & -(orbit & special)).bit_length() - 1, True
    last = ordinary.bit_length() - 1
    return taken, last + lens[last], False


def test_pointer_jumping_chain_equals_sequential_walk():
    rng = random.Random(20261018)
    for _ in range(20000):
        top = rng.choice([1, 3, 9, 12, 23])
        lens = [0 if rng.random() < 0.04 else rng.randint(1, top) for _ in range(64)]
        budget = rng.randint(1, 50)
        assert jumping(lens, budget) == sequential(lens, budget), (lens, budget)
