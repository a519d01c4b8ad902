"""BASELINE.json configurations and their synthetic inputs.

Every value comes from a splitmix64 stream (seeded per config / column) so the
GPU path and the CPU oracle see identical inputs:

* ints uniform over the full range, float64 = raw random 64-bit patterns
  (NaN payloads included; encode copies bits, access/put.go:130-134),
  bool = bit 0, string bytes printable ASCII 0x20-0x7E, bytes uniform.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Dict, Optional

import numpy as np

from .columns import HostColumns, column_specs
from .schema import (SBool, SBytes, SFloat64, SInt16, SInt32, SInt64, SMapSorted, SString,
                     SStringLen, SVariableBytes, SVariableString, SchemaChain, SchemaNamedChain,
                     SChain)

GOLDEN_GAMMA = np.uint64(0x9E3779B97F4A7C15)


def splitmix64(seed: int, count: int, start: int = 0) -> np.ndarray:
    """splitmix64 outputs z_{start+1}..z_{start+count} for state `seed`
    (counter-based: any slice of the stream is generated directly)."""
    with np.errstate(over="ignore"):
        k = np.arange(start + 1, start + count + 1, dtype=np.uint64)
        z = np.uint64(seed) + k * GOLDEN_GAMMA
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def random_bytes(seed: int, nbytes: int, byte_off: int = 0) -> np.ndarray:
    """Bytes [byte_off, byte_off + nbytes) of the little-endian splitmix64
    byte stream of `seed`; generated in bounded pieces (large shards)."""
    out = np.empty(nbytes, dtype=np.uint8)
    piece = 1 << 28
    done = 0
    while done < nbytes:
        m = min(piece, nbytes - done)
        b0 = byte_off + done
        w0 = b0 // 8
        w1 = (b0 + m + 7) // 8
        words = splitmix64(seed, w1 - w0, start=w0)
        out[done:done + m] = words.view(np.uint8)[b0 - 8 * w0: b0 - 8 * w0 + m]
        done += m
    return out


def _col_seed(seed: int, c: int) -> int:
    return (seed + (c + 1) * 0x1000_0000_0000) & 0xFFFF_FFFF_FFFF_FFFF


@dataclass
class Config:
    name: str
    chain: SchemaChain
    n: int
    seed: int
    mode: int = 0
    var_len: Optional[Callable] = None   # (n, seed, lo) -> dict col -> lengths of blobs [lo, lo + n)
    note: str = ""
    per_gpu: int = 0                     # blobs one GPU encodes in bench.py (0: n)

    @property
    def shard(self) -> int:
        return self.per_gpu or self.n


def fixed_columns(chain: SchemaChain, n: int, seed: int, var_lengths: Optional[Dict[int, np.ndarray]] = None,
                  lo: int = 0, var_base: Optional[Dict[int, int]] = None) -> HostColumns:
    """Synthetic HostColumns (no nils) for blobs [lo, lo + n) of the global
    batch of `seed`: row i of every column depends only on the global blob
    index, so the shards of a batch concatenate to the unsharded batch.
    `var_base[c]` = arena bytes of var column c before blob lo."""
    hc = HostColumns(chain, n)
    for c, sp in enumerate(hc.specs):
        node = sp.node
        s = _col_seed(seed, c)
        if sp.fixed:
            raw = random_bytes(s, n * sp.width, byte_off=lo * sp.width)
            if node.kind == "bool":
                raw &= 1
            elif node.kind == "string":
                raw = (0x20 + (raw % 95)).astype(np.uint8)
            hc.data[c] = raw
        elif sp.var:
            lens = var_lengths[c] if var_lengths and c in var_lengths else np.zeros(n, np.uint32)
            lens = np.asarray(lens, dtype=np.uint64)
            offs = np.zeros(n + 1, dtype=np.uint64)
            np.cumsum(lens, out=offs[1:])
            if offs[-1] >= 2 ** 32:
                raise ValueError("var column arena exceeds uint32 offsets; shard the batch")
            base = int(var_base.get(c, 0)) if var_base else 0
            raw = random_bytes(s, int(offs[-1]), byte_off=base)
            if node.kind == "string":
                np.remainder(raw, 95, out=raw)
                raw += 0x20
            hc.data[c] = raw
            hc.offsets[c] = offs.astype(np.uint32)
        elif sp.has_valid:
            hc.valid[c] = None  # containers always present in the configs
    return hc


# ---- schemas -------------------------------------------------------------------
# Metric M: 1M x 256 B fixed-schema tuples (8 fields, H = 18, payload 238)
CHAIN_M = SChain(SInt16, SInt32, SInt64, SFloat64, SBool, SStringLen(96), SStringLen(64), SBytes(55))
# C1: README template (int16, bool, string[2], bytes[2]) -> 17 B
CHAIN_C1 = SChain(SInt16, SBool, SStringLen(2), SBytes(2))
# C2: put_bench primitives subset: int16, int64, bool, string[24], bytes[17] -> 64 B
CHAIN_C2 = SChain(SInt16, SInt64, SBool, SStringLen(24), SBytes(17))
# C3: schema-guided named chain (names stripped on the wire)
CHAIN_C3 = SchemaNamedChain((SInt32, SInt64, SFloat64, SBool, SString, SStringLen(8), SBytes(16)),
                            ("id", "ts", "score", "flag", "label", "code", "digest"))
# C4: outer tuple with one nested PackMapSorted{kid1,kid2,role,user -> string[24]} -> 256 B
CHAIN_C4 = SChain(SInt16, SInt64, SBool, SStringLen(103),
                  SMapSorted(SString.Match("user"), SStringLen(24), SString.Match("role"), SStringLen(24),
                             SString.Match("kid2"), SStringLen(24), SString.Match("kid1"), SStringLen(24)))
# C5: mixed 64 B - 4 KB blobs
CHAIN_C5 = SChain(SInt16, SInt64, SBool, SVariableString(), SVariableBytes())


def c3_lengths(n: int, seed: int, lo: int = 0) -> Dict[int, np.ndarray]:
    r = splitmix64(seed ^ 0xC3C3, n, start=lo)
    return {4: (8 + (r % np.uint64(33))).astype(np.uint32)}  # column 4 = SString, 8..40 B


def c5_lengths(n: int, seed: int, lo: int = 0) -> Dict[int, np.ndarray]:
    """Blob size log-uniform in [64, 4096]: B = 12 (H) + 11 + ls + lb."""
    r = splitmix64(seed ^ 0xC5C5, n, start=lo).astype(np.float64) / 2.0 ** 64
    B = np.floor(np.exp(np.log(64.0) + r * (np.log(4096.0) - np.log(64.0)))).astype(np.int64)
    B = np.clip(B, 64, 4096)
    rest = B - 23
    ls = rest // 2
    lb = rest - ls
    return {3: ls.astype(np.uint32), 4: lb.astype(np.uint32)}


def x1_lengths(n: int, seed: int, lo: int = 0) -> Dict[int, np.ndarray]:
    """Blob size log-uniform in [2 KiB, 64 KiB] (B = 12 (H) + 8 + ls + lb):
    about three quarters of the blobs pass 8191 bytes."""
    r = splitmix64(seed ^ 0x1111, n, start=lo).astype(np.float64) / 2.0 ** 64
    B = np.floor(np.exp(np.log(2048.0) + r * (np.log(65536.0) - np.log(2048.0)))).astype(np.int64)
    rest = np.clip(B, 2048, 65536) - 20
    ls = rest // 3
    return {1: ls.astype(np.uint32), 2: (rest - ls).astype(np.uint32)}


# X1 (beyond BASELINE.json): ADR-001 extended containers, PACKOS_MODE_EXTENDED
CHAIN_X1 = SChain(SInt64, SVariableString(), SVariableBytes())
MODE_EXTENDED = 0x100

CONFIGS = {
    "M": Config("M", CHAIN_M, 1 << 20, 0x5EED0001,
                note="1M x 256 B fixed-schema tuples (metric)"),
    "C1": Config("C1", CHAIN_C1, 1000, 0x5EED0000, note="1k flat (int16,bool,string[2],bytes[2])"),
    "C2": Config("C2", CHAIN_C2, 1 << 20, 0x5EED0002, note="1M x 64 B PutAccess primitives"),
    "C3": Config("C3", CHAIN_C3, 1 << 20, 0x5EED0003, var_len=c3_lengths,
                 note="1M schema-guided records, encode+decode"),
    "C4": Config("C4", CHAIN_C4, 4 << 20, 0x5EED0004, note="4M x 256 B with nested PackMapSorted"),
    "C5": Config("C5", CHAIN_C5, 64 << 20, 0x5EED0005, var_len=c5_lengths, per_gpu=(64 << 20) // 8,
                 note="64M mixed 64 B-4 KB across 8 GPUs (one GPU = one 8,388,608-blob shard)"),
    "X1": Config("X1", CHAIN_X1, 1 << 16, 0x5EED00E1, mode=MODE_EXTENDED, var_len=x1_lengths,
                 note="64k blobs of 2-64 KiB, extended containers (ADR-001, beyond BASELINE)"),
}


def var_prefix(cfg: Config, lo: int, seed: Optional[int] = None) -> Dict[int, int]:
    """Arena bytes of every var column before global blob `lo`."""
    seed = cfg.seed if seed is None else seed
    base: Dict[int, int] = {}
    if not cfg.var_len or lo == 0:
        return base
    step = 1 << 22
    for a in range(0, lo, step):
        for c, l in cfg.var_len(min(step, lo - a), seed, a).items():
            base[c] = base.get(c, 0) + int(np.asarray(l, dtype=np.uint64).sum())
    return base


def make_columns(cfg: Config, n: Optional[int] = None, seed: Optional[int] = None, lo: int = 0) -> HostColumns:
    """Blobs [lo, lo + n) of config `cfg`'s synthetic batch."""
    n = cfg.n if n is None else n
    seed = cfg.seed if seed is None else seed
    vl = cfg.var_len(n, seed, lo) if cfg.var_len else None
    return fixed_columns(cfg.chain, n, seed, vl, lo=lo, var_base=var_prefix(cfg, lo, seed))


def global_blob_sizes(cfg: Config, n_global: int, static_size: int, seed: Optional[int] = None) -> np.ndarray:
    """Encoded size of every blob of a global batch of the config (no nils:
    the schema's static bytes + the var lengths), for shard planning."""
    seed = cfg.seed if seed is None else seed
    sizes = np.full(n_global, static_size, dtype=np.int64)
    if cfg.var_len:
        for c, l in cfg.var_len(n_global, seed, 0).items():
            sizes += np.asarray(l, dtype=np.int64)
    return sizes


def algorithmic_bytes(hc: HostColumns, total_out: int, with_offsets: bool) -> int:
    """bytes_in + bytes_out: value bytes + 4 B/var offset read,
    blob bytes written (+8 B per blob offset when emitted)."""
    tin = 0
    for c, sp in enumerate(hc.specs):
        if sp.fixed:
            tin += hc.n * sp.width
        elif sp.var:
            tin += int(hc.offsets[c][-1]) + 4 * hc.n
    return tin + total_out + (8 * hc.n if with_offsets else 0)
