"""Golden fixtures of the 2-D Gaussian-mixture experiment (BASELINE.json configs[0]) made by the
REFERENCE itself (build container only -- /root/reference does not exist on the GPU box).

    python tests/golden/make_golden_2d.py

Executed from the reference (read-only, nothing copied into the repo): utils_2D.py imported as a
module with its two unused, absent imports stubbed (``bm3d`` :6, ``ot`` :16 -- neither is used
by the samplers), and the two sampler definitions PnP_ULA / SnoPnP_ULA taken from
sampling_2D.py's own source text (that file is a script: module-level argparse and plotting).
The driver sequence of sampling_2D.py:72-139 (seed, posterior samples, samplers, the plots'
sub-sampling draws) is replayed with the same global numpy stream.

Output: tests/golden/gmm2d_<name>_N<N>.npz (samples of both samplers and of the posterior).

``--metric_each_step`` fixture (tests/golden/gmm2d_each_step_N250.npz): the same samplers run with
compute_metric_each_step=True (sampling_2D.py:38-39, 65-66).  The reference's Wasserstein_distance
(utils_2D.py:240-244) draws two global-stream permutations per call, which is what changes the chains;
POT (``ot.dist`` / ``ot.emd2``) is absent, so the stub module provides the squared-Euclidean cost and
an exact uniform-weight EMD (an assignment problem, scipy).  The fixture therefore pins the SAMPLES of
the metric run bit for bit (the reference's own code and draws); the distance values themselves are
this stub's, i.e. parity unpinned against POT.
"""
from __future__ import annotations

import ast
import importlib.util
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def _ot_stub():
    from scipy.optimize import linear_sum_assignment
    m = types.ModuleType("ot")
    m.dist = lambda a, b: ((a[:, None, :] - b[None, :, :]) ** 2).sum(-1)

    def emd2(a, b, M):
        r, c = linear_sum_assignment(M)
        return float(M[r, c].sum() / len(r))
    m.emd2 = emd2
    return m


def load_reference():
    for name in ("bm3d", "ot"):
        m = types.ModuleType(name) if name == "bm3d" else _ot_stub()
        if name == "bm3d":
            m.bm3d = None
            m.BM3DProfile = None
        sys.modules.setdefault(name, m)
    sys.path.insert(0, REF)
    spec = importlib.util.spec_from_file_location("utils_2D", os.path.join(REF, "utils_2D.py"))
    u = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(u)
    src = open(os.path.join(REF, "sampling_2D.py")).read()
    tree = ast.parse(src)
    defs = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in ("PnP_ULA", "SnoPnP_ULA")]
    ns = dict(vars(u))
    exec(compile(ast.Module(body=defs, type_ignores=[]), "sampling_2D.py", "exec"), ns)
    return u, ns["PnP_ULA"], ns["SnoPnP_ULA"]


def main():
    u, PnP_ULA, SnoPnP_ULA = load_reference()
    for name, N in (("symetric_gaussians", 200), ("cross", 120), ("disymmetric_gaussians", 150)):
        np.random.seed(0)
        mu_list, sigma_list, pi_list = u.gaussian_mixt_example(name)
        A, sigma = np.eye(2), 1
        D = u.Theorical_MMSE(mu_list, sigma_list, pi_list)
        Y = [np.array([0, 0]), np.array([0, -2]), np.array([-6, 6])]
        post, post2 = [], []
        for y in Y:
            post.append(u.sample_posterior(A, y, sigma, N, mu_list, sigma_list, pi_list))
            post2.append(u.sample_posterior(A, y, sigma, N, mu_list, sigma_list, pi_list))
        ula = [PnP_ULA(N, Y[i], Y[i], 0.1, A, sigma, D, 0.5, 1.5) for i in range(3)]
        for i in range(3):
            np.random.permutation(ula[i])
        sno = [SnoPnP_ULA(N, Y[i], Y[i], 0.3, A, sigma, D, 2 / 3) for i in range(3)]
        for i in range(3):
            np.random.permutation(sno[i])
        den = np.array([D(np.array([a, b]), e) for a, b, e in ((0.3, -1.2, 0.5), (4.0, 4.5, 0.3), (-6, 6, 0.1))])
        out = {f"ula{i}": ula[i] for i in range(3)}
        out.update({f"sno{i}": sno[i] for i in range(3)})
        out.update({f"post{i}": post[i] for i in range(3)})
        out.update({f"post2_{i}": post2[i] for i in range(3)})
        out["denoiser_probe"] = den
        out["next_uniform"] = np.random.rand(4)     # the stream position after the samplers
        fn = os.path.join(HERE, f"gmm2d_{name}_N{N}.npz")
        np.savez_compressed(fn, **out)
        print("wrote", fn)


def main_each_step():
    u, PnP_ULA, SnoPnP_ULA = load_reference()
    name, N = "symetric_gaussians", 250
    np.random.seed(0)
    mu_list, sigma_list, pi_list = u.gaussian_mixt_example(name)
    A, sigma = np.eye(2), 1
    D = u.Theorical_MMSE(mu_list, sigma_list, pi_list)
    Y = [np.array([0, 0]), np.array([0, -2]), np.array([-6, 6])]
    post, post2 = [], []
    for y in Y:
        post.append(u.sample_posterior(A, y, sigma, N, mu_list, sigma_list, pi_list))
        post2.append(u.sample_posterior(A, y, sigma, N, mu_list, sigma_list, pi_list))
    out = {}
    for i in range(3):
        xs, ws = PnP_ULA(N, Y[i], Y[i], 0.1, A, sigma, D, 0.5, 1.5, Sample_posterior=post[i],
                         compute_metric_each_step=True)
        out[f"ula{i}"], out[f"wula{i}"] = xs, np.array(ws)
    for i in range(3):
        np.random.permutation(out[f"ula{i}"])
    for i in range(3):
        xs, ws = SnoPnP_ULA(N, Y[i], Y[i], 0.3, A, sigma, D, 2 / 3, Sample_posterior=post[i],
                            compute_metric_each_step=True)
        out[f"sno{i}"], out[f"wsno{i}"] = xs, np.array(ws)
    for i in range(3):
        np.random.permutation(out[f"sno{i}"])
    out["next_uniform"] = np.random.rand(4)
    fn = os.path.join(HERE, f"gmm2d_each_step_N{N}.npz")
    np.savez_compressed(fn, **out)
    print("wrote", fn)


if __name__ == "__main__":
    if "--metric_each_step" in sys.argv:
        main_each_step()
    else:
        main()
