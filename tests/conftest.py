import glob
import importlib.util
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
if os.path.join(ROOT, "tests") not in sys.path:
    sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libcovt on the device)")


def load_covt():
    """Import the product package (directory name has a dash) as `covtiles_amd`."""
    if "covtiles_amd" in sys.modules:
        return sys.modules["covtiles_amd"]
    path = os.path.join(ROOT, "cov-tiles_amd", "__init__.py")
    spec = importlib.util.spec_from_file_location("covtiles_amd", path,
                                                  submodule_search_locations=[os.path.dirname(path)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["covtiles_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="session")
def covt():
    return load_covt()


@pytest.fixture(scope="session")
def oracle():
    import oracle as O

    O.build()
    return O


def tile_paths(sets=("omt", "bing", "amazon")):
    out = []
    for s in sets:
        out += sorted(glob.glob(os.path.join(GOLDEN, "tiles", s, "*.covt")))
    return out


def tile_key(path):
    return os.path.basename(os.path.dirname(path)) + "/" + os.path.basename(path)[:-5]


@pytest.fixture(scope="session")
def golden_streams():
    with open(os.path.join(GOLDEN, "oracle_streams.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def decodable_tiles(golden_streams):
    """(key, bytes) of the 126 tiles whose every Id/Geometry stream decodes."""
    res = []
    for p in tile_paths():
        k = tile_key(p)
        if golden_streams["tiles"][k]["decodable"]:
            res.append((k, open(p, "rb").read()))
    return res


@pytest.fixture(scope="session")
def gpu_available():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    return True
