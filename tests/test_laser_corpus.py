"""The LASER-shaped corpus derived from the reference's runtime bytecode
(tests/golden/laser, made by tools/make_laser_corpus.py over
tests/laser_concolic.py).

CPU checks: the committed files are exactly what the generator produces
(deterministic; one scenario re-run here), every query lowers to the engine's
vocabulary, and every witness the engine finds on the host build of the
interpreter satisfies the ORIGINAL formula under the oracle.
tests/test_gpu_laser.py runs the same corpus on the device at C2's 2^24."""
import gzip
import json
import os
import sys

import pytest

from mythril_amd.compiler import Unsupported
from mythril_amd.engine import WitnessEngine, prepare
from mythril_amd.smt2 import parse_file
from tests.fakedev import FakeDevice
from tests.test_engine_cpu import holds

HERE = os.path.dirname(os.path.abspath(__file__))
CORPUS = os.path.join(HERE, "golden", "laser")
MANIFEST = json.load(open(os.path.join(CORPUS, "manifest.json")))


def test_manifest_matches_files():
    files = {f for f in os.listdir(CORPUS) if f.endswith(".smt2.gz")}
    assert files == {m["file"] for m in MANIFEST}
    assert len(MANIFEST) >= 100
    contracts = {m["contract"] for m in MANIFEST}
    assert contracts == {"underflow", "overflow", "metacoin", "suicide"}
    assert sum(m["status"] == "sat" for m in MANIFEST) >= 50
    # multi-transaction sets carry one sender-among-actors constraint per transaction
    last = max(MANIFEST, key=lambda m: (m["tx"], m["conjuncts"]))
    text = gzip.open(os.path.join(CORPUS, last["file"]), "rt").read()
    for t in range(1, last["tx"] + 1):
        assert f"(= |sender_{t}| #x000000000000000000000000deadbeef" in text


def test_generator_is_deterministic(tmp_path):
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))
    from make_laser_corpus import write
    made = write(str(tmp_path), only="suicide/t2_kill")
    assert made
    for m in made:
        a = open(os.path.join(tmp_path, m["file"]), "rb").read()
        b = open(os.path.join(CORPUS, m["file"]), "rb").read()
        assert a == b, m["file"]


def test_every_query_lowers():
    for m in MANIFEST:
        s = parse_file(os.path.join(CORPUS, m["file"]))
        try:
            prepare(s.asserts, s.ctx)
        except Unsupported as e:   # pragma: no cover - a regression
            pytest.fail(f"{m['file']}: {e}")


def test_host_witnesses_are_sound():
    eng = WitnessEngine(dev=FakeDevice(chunk=4096), seed=0x5EED0002, budget=1 << 12)
    found = {"sat": 0, "unknown": 0}
    for m in MANIFEST:
        s = parse_file(os.path.join(CORPUS, m["file"]))
        q = prepare(s.asserts, s.ctx)
        (w,) = eng.search([q])
        if w is not None:
            assert holds(s.asserts, w), m["file"]
            found[m["status"]] += 1
    assert found["sat"] >= 40, found
