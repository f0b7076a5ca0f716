"""CPU checks of the LLC4320 source restatement (oracle.llc_load_file / get_tiles)
against digests of the reference's own SWOTRawDataLoader.load_file / get_tiles
outputs on the same synthetic full-size LLC4320 inputs (tests/llc_synth.py,
tests/golden/make_golden_llc.py).  Bit-exact: pure data movement."""
import hashlib
import json
import os

import numpy as np
import pytest

import llc_synth
from oracle import rcan_oracle as ro


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float32).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def llc():
    tmpl = llc_synth.template()
    return tmpl, [llc_synth.wet_values(tmpl, k) for k in range(2)]


def test_llc_load_file_and_get_tiles_match_reference(golden_dir, llc):
    g = json.load(open(os.path.join(golden_dir, "llc.json")))
    tmpl, vals = llc
    fields = []
    for k, gv in enumerate(g["vars"]):
        f = ro.llc_load_file(tmpl, vals[k], g["roi"], g["nx"])
        assert list(f.shape) == gv["shape"] and int(np.isnan(f).sum()) == gv["nan"]
        assert digest(f) == gv["sha256"]
        fields.append(f)
    tiles, ids, grid = ro.get_tiles(fields, 192, 192)
    assert list(tiles.shape) == g["tiles"]["shape"] and digest(tiles) == g["tiles"]["sha256"]
    assert list(ids) == g["tiles"]["tile_ids"] and grid == (g["tiles"]["grid"]["y"], g["tiles"]["grid"]["x"])


def test_llc_value_count_mismatch_raises(llc):
    tmpl, vals = llc
    with pytest.raises(ValueError):
        ro.llc_load_file(tmpl, vals[0][:-1], llc_synth.ROI)
