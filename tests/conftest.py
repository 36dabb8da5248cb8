import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a real MI355X (HIP) GPU')
    config.addinivalue_line('markers', 'slow: takes more than a few seconds')


@pytest.fixture(autouse=True)
def _loop_errors_clean():
    """Exceptions escaping loop callbacks would crash the Node reference;
    fail the test that caused them."""
    from zkmi.runtime.loop import default_loop
    loop = default_loop()
    before = len(loop.errors)
    yield
    new = loop.errors[before:]
    if new:
        raise AssertionError('exceptions in loop callbacks: %r' % (new,))


@pytest.fixture(scope='session')
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from zkmi.ops import _lib
    _lib.lib()            # fail loudly if the HIP library is missing
    return torch.device('cuda', 0)
