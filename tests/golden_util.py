"""Helpers turning tests/golden/vectors.json entries into schemas and rows."""
import json
import os

from packos_amd.schema import BuildChain

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "vectors.json")


def load():
    with open(GOLDEN) as f:
        return json.load(f)


def unwrap(v):
    if isinstance(v, dict):
        if set(v) == {"s"}:
            return v["s"]
        if set(v) == {"b"}:
            return bytes.fromhex(v["b"])
        if set(v) == {"f32"}:
            return v["f32"]
        return {k: unwrap(x) for k, x in v.items()}
    if isinstance(v, list):
        return [unwrap(x) for x in v]
    return v


def chain_of(schema_json):
    return BuildChain(schema_json)


MODES = {"putaccess": 0, "packable": 1}
