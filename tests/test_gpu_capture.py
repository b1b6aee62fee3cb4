"""hipGraph capture of the one-level stream forks the forward uses (net_ga.py's hyper / slice /
syntax side streams: main -> side, joined back), with liblic convolutions on both streams: the
replay must equal the eager run bit for bit.  The nested fork (a side stream forked from a side
stream) segfaults in capture_end even with plain torch kernels (tools/capture_fork_probe.py), so the
model keeps its forks one level deep."""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


@pytest.mark.parametrize("pattern", ["flat", "sibling"])
@pytest.mark.parametrize("use_lic", [False, True])
def test_capture_one_level_forks(pattern, use_lic):
    import capture_fork_probe as P
    assert P.run(pattern, use_lic, "global")
