"""2-D Gaussian-mixture experiment of the reference (sampling_2D.py, utils_2D.py): BASELINE.json
configs[0], the CPU-runnable plumbing case ("sampling_2D.py --N 1000 --name symetric_gaussians").

Restated in numpy (the reference runs it on the CPU with numpy too):
* the three mixtures of utils_2D.py:23-33, the exact MMSE denoiser of utils_2D.py:218-243, the
  posterior constants / sampler of utils_2D.py:142-175 and 98-114;
* PnP-ULA (sampling_2D.py:22-46) and SnoPnP-ULA -- the 2-D PSGLA -- (sampling_2D.py:49-70), with the
  same numpy operation order and the same consumption of the global ``np.random`` stream, so a run
  seeded like the reference (``np.random.seed(0)``, sampling_2D.py:10) reproduces its samples bit for
  bit (tests/golden/gmm2d_*.npz, made by tests/golden/make_golden_2d.py from the reference);
* the distances of sampling_2D.py:160-216.  POT (``ot``) is not installed: the exact earth-mover
  distance between two equal-size uniform point clouds with the squared-Euclidean cost
  (``ot.emd2(a=[], b=[], M=ot.dist(s1, s2))``, utils_2D.py:245-254) is an assignment problem, solved
  here exactly by scipy's ``linear_sum_assignment``; the sliced distance restates
  ``ot.sliced.sliced_wasserstein_distance`` (Gaussian random directions, sorted 1-D couplings).
  Both are *parity unpinned* against POT itself (absent), which only affects reported metrics.
"""
from __future__ import annotations

import numpy as np
import scipy.linalg as linalg
from scipy import stats
from scipy.optimize import linear_sum_assignment


def gaussian_mixt_example(name: str):
    """(mu_list, sigma_list, pi_list) of utils_2D.py:23-33."""
    if name == "symetric_gaussians":
        return [np.array([5, 5]), np.array([-5, -5])], [np.eye(2), np.eye(2)], [0.5, 0.5]
    if name == "cross":
        return [np.array([0, 0]), np.array([0, 0])], [[[2, 0.5], [0.5, 0.15]], [[0.15, 0.5], [0.5, 2.]]], [0.5, 0.5]
    if name == "disymmetric_gaussians":
        return [np.array([0, 3]), np.array([0, -5])], [np.eye(2), np.eye(2) / 5], [0.5, 0.5]
    raise ValueError(f"unknown mixture {name!r}")


def theoretical_mmse(mu_list, sigma_list, pi_list):
    """Exact MMSE denoiser D(x, eps) of the mixture prior (utils_2D.py:218-243).  Note the
    reference's noise covariance sqrt(eps) * Id (kept as is)."""
    r = len(mu_list)
    eye = np.eye(2)
    inv = [np.linalg.inv(s) for s in sigma_list]

    def denoiser(x, epsilon):
        se = np.sqrt(epsilon)
        num, den = 0, 0
        for i in range(r):
            d = x - mu_list[i]
            cov = se * eye + sigma_list[i]
            c = np.exp(-0.5 * d.T @ np.linalg.inv(cov) @ d)
            c = c / np.sqrt(np.linalg.det(cov))
            m = np.linalg.inv(eye / se + inv[i]) @ (x / se + inv[i] @ mu_list[i])
            num += c * pi_list[i] * m
            den += c * pi_list[i]
        return num / den
    return denoiser


def posterior_constants(A, y, sigma, mu_list, sigma_list, pi_list):
    """Means, covariances and weights of the mixture posterior x | y, y = A x + N(0, sigma)
    (utils_2D.py:142-167)."""
    p = len(mu_list)
    inv = [np.linalg.inv(s) for s in sigma_list]
    cinv = [inv[i] + A.T @ A / sigma for i in range(p)]
    cov = [np.linalg.inv(c) for c in cinv]
    eye = np.eye(2)
    mus = []
    w = np.zeros(p)
    for i in range(p):
        mus.append(cov[i] @ (inv[i] @ mu_list[i] + A @ y / sigma))
        sq = linalg.sqrtm(sigma_list[i])
        w[i] = pi_list[i] * np.exp(0.5 * (mus[i].T @ cinv[i] @ mus[i] - mu_list[i].T @ inv[i] @ mu_list[i]
                                          - y.T @ y / sigma)) / np.sqrt(np.linalg.det(sq @ A.T @ A @ sq + sigma * eye))
    return mus, cov, w / np.sum(w)


def sample_mixture(mu_list, sigma_list, pi_list, N: int):
    """N draws of a 2-D mixture, components in order then shuffled (utils_2D.py:98-114)."""
    roots = [linalg.sqrtm(s) for s in sigma_list]
    X = mu_list[0][:, None] + np.dot(roots[0], np.random.randn(2, int(pi_list[0] * N)))
    for i in range(1, len(mu_list)):
        Xi = mu_list[i][:, None] + np.dot(roots[i], np.random.randn(2, int(pi_list[i] * N)))
        X = np.concatenate([X, Xi], axis=1)
    return np.random.permutation(X.T)


def sample_posterior(A, y, sigma, N, mu_list, sigma_list, pi_list):
    mus, cov, w = posterior_constants(A, y, sigma, mu_list, sigma_list, pi_list)
    return sample_mixture(mus, cov, w, N)


def _data_score(y, x, A, sigma):
    return A.T @ (y - A @ x) / sigma ** 2


def pnp_ula(N, x_0, y, delta, A, sigma, denoiser, epsilon, alpha, post=None, metric_each_step=False):
    """PnP-ULA, N - 1 steps from x_0 (sampling_2D.py:22-46):
    x' = x + delta s(y|x) + alpha delta (D(x, eps) - x)/eps + sqrt(2 delta) z.
    metric_each_step (sampling_2D.py:38-39): after step i with i % 100 == 0, the Wasserstein distance
    between the chain so far and as many posterior samples (`post`); its sub-sampling draws come from
    the same global numpy stream, so the chain differs from a run without metrics, as in the reference.
    Returns X, or (X, distances) with metric_each_step."""
    X = [x_0]
    x = x_0
    W = []
    for i in range(N - 1):
        z = np.random.randn(y.shape[0])
        x = x + delta * _data_score(y, x, A, sigma) + alpha * delta * (1 / epsilon) * (denoiser(x, epsilon) - x) \
            + np.sqrt(2 * delta) * z
        X.append(x)
        if metric_each_step and i % 100 == 0:
            W.append(wasserstein2(np.array(X), post[:len(X), :]))
    return (np.array(X), W) if metric_each_step else np.array(X)


def snopnp_ula(N, x_0, y, delta, A, sigma, denoiser, alpha, post=None, metric_each_step=False):
    """SnoPnP-ULA -- the 2-D PSGLA: x' = D(x + (delta/alpha) s(y|x) + sqrt(2 delta) z, delta)
    (sampling_2D.py:49-70); metric_each_step as pnp_ula (sampling_2D.py:65-66)."""
    X = [x_0]
    x = x_0
    W = []
    for i in range(N - 1):
        z = np.random.randn(y.shape[0])
        x = denoiser(x + (delta / alpha) * _data_score(y, x, A, sigma) + np.sqrt(2 * delta) * z, delta)
        X.append(x)
        if metric_each_step and i % 100 == 0:
            W.append(wasserstein2(np.array(X), post[:len(X), :]))
    return (np.array(X), W) if metric_each_step else np.array(X)


def wasserstein2(sample1, sample2, n: int = 1000):
    """Exact EMD with the squared-Euclidean cost between two random 1000-point sub-samples
    (utils_2D.py:245-254: ot.emd2 with uniform weights); equal sizes => an assignment problem."""
    s1 = np.random.permutation(sample1)[:n]
    s2 = np.random.permutation(sample2)[:n]
    M = ((s1[:, None, :] - s2[None, :, :]) ** 2).sum(-1)
    r, c = linear_sum_assignment(M)
    return float(M[r, c].sum() / len(r))


def sliced_wasserstein(X_s, X_t, n_projections: int = 50, p: int = 2, rng=None):
    """ot.sliced.sliced_wasserstein_distance(X_s, X_t, n_projections, p) for uniform weights."""
    rng = np.random if rng is None else rng
    proj = rng.randn(X_s.shape[1], n_projections)
    proj = proj / np.sqrt(np.sum(proj ** 2, 0, keepdims=True))
    xs, xt = np.sort(X_s @ proj, 0), np.sort(X_t @ proj, 0)
    if xs.shape[0] != xt.shape[0]:        # quantile coupling for unequal sizes
        q = np.linspace(0, 1, max(xs.shape[0], xt.shape[0]))
        xs = np.quantile(xs, q, axis=0)
        xt = np.quantile(xt, q, axis=0)
    res = np.mean(np.abs(xs - xt) ** p, 0)
    return float((np.sum(res) / n_projections) ** (1.0 / p))


def mixture_density(positions, mu_list, sigma_list, weights):
    """sum_i w_i exp(-(x - mu_i)^T Sigma_i^-1 (x - mu_i)) on a (2, n) grid (utils_2D.py:121-136)."""
    vals = np.zeros(positions.shape[1])
    for i in range(len(mu_list)):
        d = positions.T - mu_list[i][None, :]
        vals += weights[i] * np.exp(-np.einsum("ni,ij,nj->n", d, np.linalg.inv(sigma_list[i]), d))
    return vals


def density_mse(sample, mus, covs, w):
    """sum (KDE(sample) - posterior)^2 over a 100 x 100 grid of [-8, 8]^2, both normalised
    (sampling_2D.py:186-212)."""
    X0, X1 = np.mgrid[-8:8:100j, -8:8:100j]
    pos = np.vstack([X0.ravel(), X1.ravel()])
    kde = stats.gaussian_kde(np.vstack([sample[:, 0], sample[:, 1]]))
    Z = np.reshape(kde(pos).T, X0.shape)
    Z = Z / np.sum(Z)
    P = np.reshape(mixture_density(pos, mus, covs, w).T, X0.shape)
    P = P / np.sum(P)
    return float(np.sum((Z - P) ** 2))


def run_experiment(name: str = "symetric_gaussians", N: int = 1000, seed: int = 0, metrics: bool = True,
                   metric_each_step: bool = False):
    """The body of sampling_2D.py:72-250 for one N (plots omitted): returns the result dict the
    reference np.saves (same keys; with metric_each_step also 'Wass_dist_ULA_list' and
    'Wass_dist_PSGLA_list', sampling_2D.py:246-248)."""
    np.random.seed(seed)
    mu_list, sigma_list, pi_list = gaussian_mixt_example(name)
    A = np.eye(2)
    sigma = 1
    eps_pnp, delta_pnp, alpha_pnp = 0.5, 0.1, 1.5
    delta_sno, alpha_sno = 0.3, 2 / 3
    D = theoretical_mmse(mu_list, sigma_list, pi_list)
    Y = [np.array([0, 0]), np.array([0, -2]), np.array([-6, 6])]
    post, post2 = [], []
    for y in Y:
        post.append(sample_posterior(A, y, sigma, N, mu_list, sigma_list, pi_list))
        post2.append(sample_posterior(A, y, sigma, N, mu_list, sigma_list, pi_list))
    wula, wsno = [], []
    if metric_each_step:
        ula = []
        for i in range(3):
            xs, ws = pnp_ula(N, Y[i], Y[i], delta_pnp, A, sigma, D, eps_pnp, alpha_pnp, post=post[i],
                             metric_each_step=True)
            ula.append(xs)
            wula.append(ws)
    else:
        ula = [pnp_ula(N, Y[i], Y[i], delta_pnp, A, sigma, D, eps_pnp, alpha_pnp) for i in range(3)]
    for i in range(3):                      # the plot's sub-sampling draws (sampling_2D.py:114)
        np.random.permutation(ula[i])
    if metric_each_step:
        sno = []
        for i in range(3):
            xs, ws = snopnp_ula(N, Y[i], Y[i], delta_sno, A, sigma, D, alpha_sno, post=post[i], metric_each_step=True)
            sno.append(xs)
            wsno.append(ws)
    else:
        sno = [snopnp_ula(N, Y[i], Y[i], delta_sno, A, sigma, D, alpha_sno) for i in range(3)]
    for i in range(3):
        np.random.permutation(sno[i])
    out = {"A": A, "mu_list": mu_list, "sigma_list": sigma_list, "pi_list": pi_list, "sigma": sigma,
           "delta_pnp_ula": delta_pnp, "delta_snopnp_ula": delta_sno, "alpha_pnp_ula": alpha_pnp,
           "alpha_snopnp_ula": alpha_sno, "epsilon_pnp_ula": eps_pnp, "Y": Y,
           "Sample_PnP_ULA": ula, "Sample_SnoPnP_ULA": sno}
    if metrics:
        keys = ["Sliced_Wass_PnP_ULA", "Sliced_Wass_SnoPnP_ULA", "Sliced_Wass_ref", "Wass_PnP_ULA",
                "Wass_SnoPnP_ULA", "Wass_ref", "MMSE_PnP_ULA", "MMSE_SnoPnP_ULA"]
        for k in keys:
            out[k] = []
        for i in range(len(Y)):
            out["Sliced_Wass_PnP_ULA"].append(sliced_wasserstein(post[i], ula[i]))
            out["Sliced_Wass_SnoPnP_ULA"].append(sliced_wasserstein(post[i], sno[i]))
            out["Sliced_Wass_ref"].append(sliced_wasserstein(post[i], post2[i]))
            out["Wass_PnP_ULA"].append(wasserstein2(post[i], ula[i]))
            out["Wass_SnoPnP_ULA"].append(wasserstein2(post[i], sno[i]))
            out["Wass_ref"].append(wasserstein2(post[i], post2[i]))
            mus, cov, w = posterior_constants(A, Y[i], sigma, mu_list, sigma_list, pi_list)
            out["MMSE_PnP_ULA"].append(density_mse(ula[i], mus, cov, w))
            out["MMSE_SnoPnP_ULA"].append(density_mse(sno[i], mus, cov, w))
    if metric_each_step:
        out["Wass_dist_ULA_list"] = wula
        out["Wass_dist_PSGLA_list"] = wsno
    return out


def main(argv=None):
    """CLI with the reference's sampling_2D.py flags (--name, --N, --metric_each_step)."""
    import argparse
    import os
    p = argparse.ArgumentParser()
    p.add_argument("--name", type=str, default="symetric_gaussians",
                   choices=["symetric_gaussians", "disymmetric_gaussians", "cross"])
    p.add_argument("--N", type=int)
    p.add_argument("--metric_each_step", type=bool, default=False)
    p.add_argument("--results_root", type=str, default="results")
    pars = p.parse_args(argv)
    path = os.path.join(pars.results_root, "result_GMM")
    os.makedirs(path, exist_ok=True)
    for N in ([100, 1000, 10000] if pars.N is None else [pars.N]):
        res = run_experiment(pars.name, N, metric_each_step=pars.metric_each_step)
        for i in range(3):
            print("Observation " + str(i))
            print("Sliced Wasserstein for PnP ULA = {:.2f} and SnoPnP ULA = {:.2f} and reference dist = {:.2f}".format(
                res["Sliced_Wass_PnP_ULA"][i], res["Sliced_Wass_SnoPnP_ULA"][i], res["Sliced_Wass_ref"][i]))
            print("Wasserstein dist for PnP ULA = {:.2f} and SnoPnP ULA = {:.2f} and reference dist = {:.2f}".format(
                res["Wass_PnP_ULA"][i], res["Wass_SnoPnP_ULA"][i], res["Wass_ref"][i]))
            print("MMSE dist for PnP ULA = {} and SnoPnP ULA = {}".format(res["MMSE_PnP_ULA"][i],
                                                                          res["MMSE_SnoPnP_ULA"][i]))
        np.save(os.path.join(path, "Sample_PnP_SnoPnP_ULA_" + pars.name + "_N" + str(N) + "_result.npy"), res,
                allow_pickle=True)
    return res


if __name__ == "__main__":
    main()
