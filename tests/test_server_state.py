"""The fused server step refuses a state without the moments its rule reads (ADVICE r3,
medium): a centered RMSProp given a plain RMSProp state (no 'm'), Adam given an SGD state.
Checked on the CPU before anything is launched: the Python guard raises ValueError and the
native one-call path (fjhost.server_pairs) declines instead of launching with a null state
table entry."""
import ctypes

import pytest
import torch

from fedjax_amd import _lib, server


@pytest.mark.parametrize("opt,state", [
    (server.rmsprop(0.1, centered=True), {"count": 0, "v": {"w": torch.zeros(3)}}),
    (server.adam(0.1), {"count": 0, "m": {"w": torch.zeros(3)}}),
    (server.adam(0.1), {"count": 0}),
    (server.sgd(0.1, momentum=0.9), {"count": 0}),
])
def test_missing_moment_raises(opt, state):
    pairs = [({"w": torch.ones(3)}, 1)]
    with pytest.raises(ValueError, match="optimizer state has no"):
        server.fused_tree_mean_update(pairs, opt, {"w": torch.zeros(3)}, state)


def test_native_server_pairs_declines_without_the_moments():
    opt = server.adam(0.1)
    desc = opt.descriptor(1)
    pairs = [({"w": torch.ones(3)}, 1)]
    got = _lib.host().server_pairs(pairs, {"w": torch.zeros(3)}, None, None, None, ctypes.addressof(desc),
                                   0.0, 0, 0)
    assert got is None


def test_plain_sgd_needs_no_moments():
    server._require_state(server.sgd(0.1), {"count": 0})
