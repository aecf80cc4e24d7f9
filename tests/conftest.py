import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (run with -m gpu)')
    config.addinivalue_line('markers', 'slow: longer CPU test')
    config.addinivalue_line('markers', 'fresh_process: starts a child Python; runs before any test touches the GPU')


@pytest.hookimpl(trylast=True)
def pytest_collection_modifyitems(session, config, items):
    # tests that start a child process run first, while this process has not
    # initialised the GPU (a child forked from a GPU process must not exec).
    # trylast: after every other plugin's reordering (--ff / --nf, random
    # orders), so this sort is the one that holds
    items.sort(key=lambda it: 0 if it.get_closest_marker('fresh_process') else 1)


def gpu_initialised():
    """whether this process has opened the GPU: /dev/kfd among its open files,
    or torch's HIP context up (a fork + exec from such a process is what the
    pool forbids)"""
    try:
        for fd in os.listdir('/proc/self/fd'):
            try:
                if os.readlink(os.path.join('/proc/self/fd', fd)) == '/dev/kfd':
                    return True
            except OSError:
                pass
    except OSError:
        pass
    torch = sys.modules.get('torch')
    try:
        return bool(torch is not None and torch.cuda.is_initialized())
    except Exception:
        return False


@pytest.fixture(autouse=True)
def _fresh_process_guard(request):
    """a fresh_process test starts a child process: refuse to run it once this
    process has touched the GPU, whatever order the tests ended up in"""
    if request.node.get_closest_marker('fresh_process') and gpu_initialised():
        pytest.skip('this process has initialised the GPU: a child process started now would fork + exec from '
                    'it (run this test on its own, or first)')
    yield


@pytest.fixture(scope='session')
def golden_dir():
    return os.path.join(REPO, 'tests', 'golden')
