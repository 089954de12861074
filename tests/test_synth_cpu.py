"""The synthetic BA windows the GPU tests and the bench run on (visionx-slam_amd/python/vxslam/synth.py):
the connected C5 rig (cross_frac, round 4) — the 8 streams form ONE covisibility component, every shared
observation projects inside the neighbouring camera's image in front of it — and cross_frac = 0 leaves
the round-3 maps unchanged."""
import numpy as np

from vxslam import synth


def _components(m):
    from scipy.sparse import coo_matrix
    from scipy.sparse.csgraph import connected_components

    row = {int(k): i for i, k in enumerate(m["kf_id"])}
    ptr, kid = m["lm_obs_ptr"], m["obs_kf_id"]
    r, c = [], []
    for l in range(len(m["lm_id"])):
        ks = [row[int(x)] for x in kid[ptr[l]:ptr[l + 1]]]
        r += [ks[0]] * (len(ks) - 1)
        c += ks[1:]
    n = len(m["kf_id"])
    return connected_components(coo_matrix((np.ones(len(r)), (r, c)), shape=(n, n)), directed=False)[0]


def test_rig_cross_frac_connects_the_streams():
    base = synth.make_ba_map(0x5EED00C5, 96, 16000, n_streams=8, n_old_kf=16)
    same = synth.make_ba_map(0x5EED00C5, 96, 16000, n_streams=8, n_old_kf=16, cross_frac=0.0)
    for k in base:
        assert np.array_equal(np.asarray(base[k]), np.asarray(same[k])), k
    assert _components(base) == 8
    m = synth.make_ba_map(0x5EED00C5, 96, 16000, n_streams=8, n_old_kf=16, cross_frac=0.03)
    assert _components(m) == 1
    assert len(m["obs_kf_id"]) > len(base["obs_kf_id"])
    # observations name their features (and back); the shared observations lie inside the neighbour's
    # image (the anchor stream's own 2-5 keyframe tracks may leave it by a few pixels, as before)
    def outside(mm):
        lm_obs = np.repeat(np.arange(len(mm["lm_id"])), np.diff(mm["lm_obs_ptr"]))
        row = {int(k): i for i, k in enumerate(mm["kf_id"])}
        ks = np.array([row[int(x)] for x in mm["obs_kf_id"]])
        f = mm["kf_feat_ptr"][ks] + mm["obs_feat_idx"].astype(np.int64)
        assert np.array_equal(mm["feat_lm_id"][f], mm["lm_id"][lm_obs])
        uv = mm["feat_uv"].reshape(-1, 2)[f]
        return int(((uv[:, 0] < 0) | (uv[:, 0] > 640) | (uv[:, 1] < 0) | (uv[:, 1] > 480)).sum())

    assert outside(m) <= outside(base)
