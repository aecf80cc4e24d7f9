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


def pytest_collection_modifyitems(session, config, items):
    # tests that start a child process run first, while this process has not
    # initialised the GPU (a child forked from a GPU process must not exec)
    items.sort(key=lambda it: 0 if it.get_closest_marker('fresh_process') else 1)


@pytest.fixture(scope='session')
def golden_dir():
    return os.path.join(REPO, 'tests', 'golden')
