import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (HIP device)')
    config.addinivalue_line('markers', 'slow: large-volume checks')


def integration_blocks():
    """The ```python blocks of INTEGRATION.md, in order (the reference-side bindings a maintainer
    would add; the tests execute them as written)."""
    import re
    txt = open(os.path.join(ROOT, 'INTEGRATION.md')).read()
    return re.findall(r'```python\n(.*?)```', txt, flags=re.S)


def exec_integration_binding():
    """Execute INTEGRATION.md section B's binding block as written, with CC_MI355X_LIB naming the
    in-tree library; returns its namespace (label_volume, _Res, _L, ...)."""
    from cluster_tools_amd import _lib
    os.environ['CC_MI355X_LIB'] = _lib.LIB_PATH
    block = [b for b in integration_blocks() if 'cc_mi355x.py' in b][0]
    ns = {'__name__': 'cc_mi355x_binding'}
    exec(compile(block, 'INTEGRATION.md#B', 'exec'), ns)
    return ns


def golden_index():
    with open(os.path.join(GOLDEN, 'index.json')) as f:
        return json.load(f)


def load_golden(name):
    d = np.load(os.path.join(GOLDEN, name + '.npz'))
    out = {k: d[k] for k in d.files}
    if 'input' not in out:
        out['input'] = out['input_q'].astype(np.float32) / np.float32(256)
    return out


@pytest.fixture(scope='session', autouse=True)
def _library_provenance():
    """On a GPU box, refuse to test a libcc_mi355x.so built from other sources than this tree's
    (cc_version() carries the source hash build.py embedded)."""
    import torch
    if torch.cuda.is_available() and not os.environ.get('CC_LIB_PATH'):   # CC_LIB_PATH: A/B builds only
        from cluster_tools_amd import _lib
        _lib.check_provenance()
    yield


@pytest.fixture(scope='session')
def ctx():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from cluster_tools_amd import _lib
    c = _lib.Context(0)
    yield c
    c.close()
