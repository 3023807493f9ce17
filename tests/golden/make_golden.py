"""Regenerates tests/golden/oracle_renders.json: tiny CPU-oracle renders, hashed.

These pin the oracle against regressions (they are self-generated, not reference truth: the reference's
GLSL kernel cannot run in this container).  Run: python tests/golden/make_golden.py
`--contract E` writes contract_e_renders.json instead: the same cases in the round-1 arithmetic contract
(oracle/srt_oracle.c ORACLE_CONTRACT 4).  Its hashes equal the oracle_renders.json of round 1 (commit
9502f3d), which tests/test_contract_tolerance.py checks, so either contract can be re-checked later.
"""
import hashlib
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "simple-ray-tracer_amd"))
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import srt_amd as S  # noqa: E402
from srt_amd import render as R  # noqa: E402
from conftest import oracle_render  # noqa: E402

CASES = [
    dict(scene="spheres", width=64, height=64, spp=2, max_depth=5),
    dict(scene="rubik", width=64, height=64, spp=2, max_depth=5),
    dict(scene="rubik", width=40, height=24, spp=3, max_depth=2),
    dict(scene="spheres", width=24, height=40, spp=3, max_depth=8),
]


def main():
    contract = sys.argv[sys.argv.index("--contract") + 1] if "--contract" in sys.argv else "A"
    out = []
    for c in CASES:
        models = [S.load_obj(ROOT / "tests/golden/objects/Rubik/Rubik.obj")] if c["scene"] == "rubik" else None
        setup = R.make_setup(c["width"], c["height"], show_model=c["scene"] == "rubik", models=models,
                             max_depth=c["max_depth"])
        acc, img, st = oracle_render(setup, c["spp"], contract=contract)
        out.append(dict(c, accum_sha256=hashlib.sha256(acc.tobytes()).hexdigest(),
                        out_sha256=hashlib.sha256(img.tobytes()).hexdigest(), rays=st["rays"]))
    name = "oracle_renders.json" if contract == "A" else f"contract_{contract.lower()}_renders.json"
    (ROOT / "tests/golden" / name).write_text(json.dumps({"cases": out}, indent=1) + "\n")


if __name__ == "__main__":
    main()
