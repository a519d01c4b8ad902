"""The cgo shim's call sequence in C (tests/c_abi_harness.c): compile a
json.Marshal-shaped SchemaJSON, pinned host columns, packos_encode_host_batch
vs the reference's bytes (access/put_test.go:12-41), packos_decode_host_batch
back.  Built by `make -C oracle harness` (__graft_entry__.build())."""
import os
import subprocess

import pytest

from golden_util import load

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "tests", "c_abi_harness")


def _want():
    return next(c["hex"] for c in load()["encode"] if c["id"] == "put_flat17")


def test_harness_built_against_libpackos():
    if not os.path.exists(HARNESS):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "harness"])
    assert os.access(HARNESS, os.X_OK)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 100_000])
def test_c_abi_harness(n):
    r = subprocess.run([HARNESS, _want(), str(n)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "c_abi_harness ok" in r.stdout
