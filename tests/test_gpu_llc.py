"""LLC4320 source -> tiles on the HIP path (srmi.llc: srmi_llc_index_map /
srmi_llc_gather / srmi_tiles_nonfinite / srmi_tiles_gather through the C ABI)
against the digests of the reference's own load_file / get_tiles outputs on the
same synthetic full-size inputs (tests/golden/llc.json).  Bit-exact."""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import llc_synth  # noqa: E402
from srmi.llc import LLCSource, get_tiles  # noqa: E402


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float32).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def files(tmp_path_factory):
    root = str(tmp_path_factory.mktemp("llc"))
    tname, dnames = llc_synth.write_files(root, 2)
    return root, tname, dnames


def test_llc_source_and_tiles_match_reference(golden_dir, files):
    g = json.load(open(os.path.join(golden_dir, "llc.json")))
    root, tname, dnames = files
    d = torch.device("cuda", 0)
    src = LLCSource(os.path.join(root, tname), roi=g["roi"], nx=g["nx"], device=d)
    fields = []
    for k, gv in enumerate(g["vars"]):
        f = src.load_file(os.path.join(root, dnames[k]))
        torch.cuda.synchronize()
        fh = f.cpu().numpy()
        assert list(fh.shape) == gv["shape"] and int(np.isnan(fh).sum()) == gv["nan"]
        assert digest(fh) == gv["sha256"]
        fields.append(f)
    region = src.load_region_data([os.path.join(root, n) for n in dnames])
    assert torch.equal(torch.nan_to_num(region[0:1], 7.0), torch.nan_to_num(fields[0], 7.0))
    tiles, ids, grid = get_tiles(region, 192, 192)
    torch.cuda.synchronize()
    assert list(tiles.shape) == g["tiles"]["shape"] and digest(tiles.cpu().numpy()) == g["tiles"]["sha256"]
    assert list(ids) == g["tiles"]["tile_ids"] and grid == (g["tiles"]["grid"]["y"], g["tiles"]["grid"]["x"])


def test_llc_wrong_value_count_raises(files):
    root, tname, dnames = files
    d = torch.device("cuda", 0)
    src = LLCSource(os.path.join(root, tname), roi=llc_synth.ROI, device=d)
    bad = os.path.join(root, "short.data")
    np.fromfile(os.path.join(root, dnames[0]), dtype=np.uint8)[:-4].tofile(bad)
    with pytest.raises(ValueError):
        src.load_file(bad)
