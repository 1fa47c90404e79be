"""Load shares of the gateway's consistent-hash ring, and worker addresses that balance it.

The gateway routes a request to the worker owning the first virtual node at or after
FNV-1a(request_id) on a 2^32 ring, 150 virtual nodes per worker named "<addr>#i"
(csrc/serve/consistent_hash.cpp, bit-identical to /root/reference/src/consistent_hash.cpp:6-45 and
/root/reference/include/consistent_hash.h:12).  FNV-1a without a finaliser places the vnodes of
"127.0.0.1:<port>#0..149" in clusters, so a ring of N workers on arbitrary ports is far from
uniform: over random port sets the busiest of 8 workers owns 1.3-2.6x its fair 1/8 (median 1.55x;
the reference's own 3-worker run split 46.8 / 24.7 / 38.5 %, /root/reference/README.md:298-300).
Consecutive decimal request ids ("r0_0000000001", ...) cluster the same way.

bench.py keeps the routing exactly as it is (parity) and changes only deployment choices:
  * the workers' ports are picked by coordinate descent over candidate ports so that the ring arcs
    are balanced (`balanced_ports`), and
  * the load generator prints request numbers scrambled (`scrambled_ids`, loadgen scramble_ids),
    which FNV-1a spreads like random ids.
`predict` reports the resulting shares for the bench's actual ids (docs/DESIGN.md §7 table).
"""
from __future__ import annotations

import random
from typing import Dict, Iterable, List, Sequence

import numpy as np

VNODES = 150
RING = 1 << 32


def _fnv(s: str) -> int:
    from .. import native

    return native.fnv1a(s)


def vnode_hashes(name: str, vnodes: int = VNODES) -> np.ndarray:
    return np.array([_fnv("%s#%d" % (name, i)) for i in range(vnodes)], np.int64)


def arc_shares_from_hashes(hs: Sequence[np.ndarray]) -> np.ndarray:
    """Fraction of the hash space each node owns (a key goes to the first vnode >= its hash,
    wrapping; on equal vnode hashes the later-added node wins, as std::map assignment does)."""
    h = np.concatenate(hs)
    own = np.concatenate([np.full(len(x), j) for j, x in enumerate(hs)])
    o = np.lexsort((-np.arange(len(h)), h))  # sort by hash; among equal hashes the last added first
    h, own = h[o], own[o]
    keep = np.concatenate([[True], h[1:] != h[:-1]])  # duplicate vnode hashes: the ring keeps one
    h, own = h[keep], own[keep]
    arcs = np.diff(np.concatenate([[h[-1] - RING], h]))
    return np.bincount(own, weights=arcs, minlength=len(hs)) / RING


def arc_shares(names: Sequence[str], vnodes: int = VNODES) -> np.ndarray:
    return arc_shares_from_hashes([vnode_hashes(n, vnodes) for n in names])


def balanced_ports(world: int, candidates: Iterable[int], seed: int = 0, rounds: int = 3, tries: int = 600,
                   host: str = "127.0.0.1") -> List[int]:
    """`world` ports from `candidates` whose "host:port" ring has balanced arcs (coordinate descent:
    each position in turn takes the candidate that lowers the largest share most)."""
    cands = list(candidates)
    if world <= 1:
        return cands[:world]
    rng = random.Random(seed)
    cache: Dict[int, np.ndarray] = {}

    def hv(p):
        if p not in cache:
            cache[p] = vnode_hashes("%s:%d" % (host, p))
        return cache[p]

    sel = rng.sample(cands, world)
    best = arc_shares_from_hashes([hv(p) for p in sel]).max()
    for _ in range(rounds):
        for j in range(world):
            for p in rng.sample(cands, min(tries, len(cands))):
                if p in sel:
                    continue
                trial = sel[:j] + [p] + sel[j + 1:]
                m = arc_shares_from_hashes([hv(q) for q in trial]).max()
                if m < best:
                    best, sel = m, trial
    return sel


def splitmix64(x: int) -> int:
    M = (1 << 64) - 1
    x = (x + 0x9E3779B97F4A7C15) & M
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M
    return x ^ (x >> 31)


_HALF = 10 ** 5


def scramble_id(i: int) -> int:
    """A bijection of [0, 10^10) (csrc/serve/loadgen.cpp scramble_id): a 4-round Feistel network on
    the two 5-digit halves with splitmix64 round functions -- distinct request numbers stay distinct
    (splitmix64(i) % 10^10 collided a few times in a few hundred thousand ids) and their
    decimal strings spread over the FNV-1a ring like random ids."""
    left, right = divmod(i % 10 ** 10, _HALF)
    for k in range(4):
        left, right = right, (left + splitmix64(right * 4 + k) % _HALF) % _HALF
    return left * _HALF + right


def request_ids(prefix: str, n: int, scramble: bool = True) -> List[str]:
    """The ids csrc/serve/loadgen.cpp sends: prefix + 10 digits (scrambled: scramble_id(i))."""
    return [prefix + "%010d" % (scramble_id(i) if scramble else i) for i in range(n)]


def reference_layout(world: int, n: int) -> Dict[str, object]:
    """What the reference's own deployment would route: workers on consecutive ports from 8001
    (/root/reference/README.md:103-109) and sequential ids "req_<i>" (/root/reference/benchmark.py:22),
    i.e. the ring without bench.py's port choice and id scramble."""
    names = ["127.0.0.1:%d" % (8001 + k) for k in range(world)]
    return dict(predict(names, ["req_%d" % i for i in range(n)]), ports=[8001 + k for k in range(world)],
                ids="req_<i>, sequential")


def route_shares(names: Sequence[str], ids: Iterable[str]) -> np.ndarray:
    """Measured-equivalent shares: route every id through the native ring (the gateway's code)."""
    from .. import native

    ring = native.Ring(VNODES)
    for n in names:
        ring.add(n)
    idx = {n: i for i, n in enumerate(names)}
    cnt = np.zeros(len(names))
    for k in ids:
        cnt[idx[ring.get(k)]] += 1
    return cnt / max(1.0, cnt.sum())


def predict(names: Sequence[str], ids: Sequence[str]) -> Dict[str, object]:
    """Shares for the given ids, the largest over the fair share, and the scaling efficiency a
    closed loop limited by its busiest worker can reach (fair / largest)."""
    s = route_shares(names, ids)
    fair = 1.0 / len(names)
    return {"shares": [round(float(x), 4) for x in s], "max_over_fair": round(float(s.max() / fair), 3),
            "efficiency": round(float(fair / s.max()), 3)}
