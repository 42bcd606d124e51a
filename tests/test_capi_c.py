"""The C ABI from a plain C program (tests/capi/capi_golden.c): no Python or
torch in the evaluating process, the way a Rust FFI consumer would link
libfnnue.so.  The committed golden vectors (tests/golden/golden_evals.json)
are written to a text fixture the program reads."""
import json
import os
import subprocess

import pytest

from tests.conftest import ROOT

CAPI = os.path.join(ROOT, "tests", "capi")
EXE = os.path.join(CAPI, "capi_golden")


def _binary() -> str:
    if not os.path.exists(EXE):  # normally built by __graft_entry__.build()
        subprocess.run(["make", "-C", CAPI, "-s"], check=True)
    return EXE


def test_c_binary_links_and_loads():
    """The program links against libfnnue.so (+ librccl, libamdhip64) and starts
    without Python; no arguments -> usage, exit 2 (no GPU call)."""
    r = subprocess.run([_binary()], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "usage" in r.stderr


@pytest.mark.gpu
def test_c_consumer_golden_vectors(tmp_path):
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "golden_evals.json")))
    lines = [str(len(g["nets"]))]
    for net in g["nets"]:
        lines.append(f"{net['seed']} {net['hd']} {net['flags']} {net['file_hash']} {len(g['positions_hex'])}")
        for h, ps, po in zip(g["positions_hex"], net["psqt"], net["positional"]):
            lines.append(f"{h} {ps} {po}")
    fx = tmp_path / "golden.txt"
    fx.write_text("\n".join(lines) + "\n")
    r = subprocess.run([_binary(), str(fx)], capture_output=True, text=True, timeout=120)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip().endswith("ok")
