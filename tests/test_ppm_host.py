"""Host-side logic of the sharded PPM update pass (no GPU): the merge by hit-point owner that
ceng795_amd.ppm.merge_shard_states performs for one-process-per-GPU runs."""
import numpy as np
import pytest

from ceng795_amd import ppm


def test_merge_takes_each_hit_point_from_its_owner():
    rng = np.random.default_rng(3)
    n, shards = 1000, 3
    states = [rng.random((n, 5), dtype=np.float32) for _ in range(shards)]
    owners = rng.integers(0, shards, n).astype(np.int32)
    got = ppm.merge_shard_states(states, owners)
    for h in range(0, n, 37):
        assert np.array_equal(got[h], states[owners[h]][h])
    assert got.dtype == np.float32 and got.shape == (n, 5)


def test_merge_rejects_bad_owners():
    states = [np.zeros((4, 5), np.float32)] * 2
    with pytest.raises(ValueError):
        ppm.merge_shard_states(states, np.array([0, 1, 2, 0]))
    with pytest.raises(ValueError):
        ppm.merge_shard_states(states, np.array([0, 1, 0]))
