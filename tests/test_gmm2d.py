"""BASELINE.json configs[0] (sampling_2D.py, CPU): the numpy restatement against fixtures made by the
reference's own samplers (tests/golden/make_golden_2d.py) -- bit for bit, same global numpy stream."""
import os

import numpy as np
import pytest

from psgla_for_posterior_sampling_amd import gmm2d

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("name,N", [("symetric_gaussians", 200), ("cross", 120), ("disymmetric_gaussians", 150)])
def test_samplers_match_reference(name, N):
    fx = dict(np.load(os.path.join(G, f"gmm2d_{name}_N{N}.npz"), allow_pickle=False))
    res = gmm2d.run_experiment(name, N, seed=0, metrics=False)
    for i in range(3):
        np.testing.assert_array_equal(res["Sample_PnP_ULA"][i], fx[f"ula{i}"])
        np.testing.assert_array_equal(res["Sample_SnoPnP_ULA"][i], fx[f"sno{i}"])
    np.testing.assert_array_equal(np.random.rand(4), fx["next_uniform"])
    mu, sg, pi = gmm2d.gaussian_mixt_example(name)
    D = gmm2d.theoretical_mmse(mu, sg, pi)
    probe = np.array([D(np.array([a, b]), e) for a, b, e in ((0.3, -1.2, 0.5), (4.0, 4.5, 0.3), (-6, 6, 0.1))])
    np.testing.assert_array_equal(probe, fx["denoiser_probe"])


def test_posterior_sampler_matches_reference():
    fx = dict(np.load(os.path.join(G, "gmm2d_symetric_gaussians_N200.npz"), allow_pickle=False))
    np.random.seed(0)
    mu, sg, pi = gmm2d.gaussian_mixt_example("symetric_gaussians")
    for i, y in enumerate([np.array([0, 0]), np.array([0, -2]), np.array([-6, 6])]):
        np.testing.assert_array_equal(gmm2d.sample_posterior(np.eye(2), y, 1, 200, mu, sg, pi), fx[f"post{i}"])
        np.testing.assert_array_equal(gmm2d.sample_posterior(np.eye(2), y, 1, 200, mu, sg, pi), fx[f"post2_{i}"])


def test_distances_behave():
    rng = np.random.RandomState(3)
    a = rng.randn(500, 2)
    assert gmm2d.wasserstein2(a, a.copy(), n=500) == 0.0
    b = a + np.array([3.0, 0.0])
    # translation by t: W2^2 = |t|^2 exactly, sliced W2 = sqrt(E_theta <t, theta>^2) ~ |t| / sqrt(2)
    assert abs(gmm2d.wasserstein2(a, b, n=500) - 9.0) < 1e-9
    assert 1.5 < gmm2d.sliced_wasserstein(a, b, n_projections=400) < 2.7


def test_cli_writes_result(tmp_path):
    res = gmm2d.main(["--N", "100", "--results_root", str(tmp_path)])
    f = tmp_path / "result_GMM" / "Sample_PnP_SnoPnP_ULA_symetric_gaussians_N100_result.npy"
    assert f.exists()
    d = np.load(f, allow_pickle=True).item()       # written by this test
    assert set(res) == set(d) and len(d["Sample_SnoPnP_ULA"]) == 3 and d["Sample_PnP_ULA"][0].shape == (100, 2)


def test_metric_each_step_matches_reference():
    """--metric_each_step (sampling_2D.py:38-39, 65-66): the per-100-step Wasserstein calls draw from
    the global numpy stream, so the chains differ from a plain run; the samples of that run match the
    reference's own samplers bit for bit (tests/golden/make_golden_2d.py --metric_each_step).  The
    distance values use the same exact EMD on both sides (POT is absent: parity unpinned against it)."""
    fx = dict(np.load(os.path.join(G, "gmm2d_each_step_N250.npz"), allow_pickle=False))
    res = gmm2d.run_experiment("symetric_gaussians", 250, seed=0, metrics=False, metric_each_step=True)
    for i in range(3):
        np.testing.assert_array_equal(res["Sample_PnP_ULA"][i], fx[f"ula{i}"])
        np.testing.assert_array_equal(res["Sample_SnoPnP_ULA"][i], fx[f"sno{i}"])
        assert len(res["Wass_dist_ULA_list"][i]) == 3 and len(res["Wass_dist_PSGLA_list"][i]) == 3
        np.testing.assert_allclose(res["Wass_dist_ULA_list"][i], fx[f"wula{i}"], rtol=1e-12)
        np.testing.assert_allclose(res["Wass_dist_PSGLA_list"][i], fx[f"wsno{i}"], rtol=1e-12)
    np.testing.assert_array_equal(np.random.rand(4), fx["next_uniform"])
