"""Order-independent 64-bit hashes for full-size parity fixtures -- TEST
INFRASTRUCTURE.  Both sides (the oracle when the fixture is made, the HIP
engine when it is checked) hash their records the same way:

* a record (a row of uint64 words) hashes by a splitmix64 chain over its words;
* a host's trace multiset hashes to the sum (mod 2^64) of its records' hashes,
  so the order the records were written in does not matter;
* a block of host digests hashes by chaining the hosts' hashes in host order.
"""
import numpy as np

_G = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def mix64(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        x ^= x >> np.uint64(30)
        x *= _M1
        x ^= x >> np.uint64(27)
        x *= _M2
        x ^= x >> np.uint64(31)
    return x


def row_hash(words: np.ndarray) -> np.ndarray:
    """[N, K] uint64 -> [N] uint64."""
    words = np.ascontiguousarray(words, dtype=np.uint64)
    h = np.zeros(words.shape[0], np.uint64)
    with np.errstate(over="ignore"):
        for k in range(words.shape[1]):
            h = mix64(h ^ (words[:, k] + _G * np.uint64(k + 1)))
    return h


def trace_host_hashes(tr: np.ndarray, n_hosts: int) -> np.ndarray:
    """Per host, the multiset hash of the trace records it logged ([n_hosts] uint64)."""
    rh = row_hash(np.ascontiguousarray(tr).view(np.uint64).reshape(len(tr), 4))
    out = np.zeros(n_hosts, np.uint64)
    np.add.at(out, tr["host"].astype(np.int64), rh)
    return out


def digest_block_hashes(dg: np.ndarray, block: int) -> np.ndarray:
    """Hashes of consecutive blocks of `block` host digests."""
    hh = row_hash(np.ascontiguousarray(dg).view(np.uint64).reshape(len(dg), -1))
    nb = (len(hh) + block - 1) // block
    pad = np.zeros(nb * block, np.uint64)
    pad[:len(hh)] = hh
    cols = pad.reshape(nb, block)
    n_in = np.minimum(block, len(hh) - np.arange(nb) * block)   # hosts in each block
    out = np.zeros(nb, np.uint64)
    for j in range(block):
        nxt = mix64(out ^ cols[:, j])
        out = np.where(j < n_in, nxt, out)
    return out
