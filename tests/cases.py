"""Seeded test cases: packed base sets + cluster posteriors + E-step constants.

Base HMMs come from the product's synthetic generator (same generator the
bench uses, on the CPU); cluster posteriors from the 'baseem' initialisation,
then perturbed so that every cluster/state has distinct transition, prior,
precision and scale parameters (baseem alone gives uniform epsilon/eta, which
would leave logA constant and hide indexing errors).
"""
from __future__ import annotations

import numpy as np

import pkgload
import vbhem_oracle as vo

vb = pkgload.load()


def post_dict(post) -> dict:
    return {k: (np.array(v) if isinstance(v, np.ndarray) else v) for k, v in post.asdict().items()}


def make_case(N=6, K=3, S=3, Sb=3, d=2, covmode=1, seed=0, ragged=False, perturb=True,
              tau=10, exprmt1=False, face=False, Nv=100, **opt_over):
    """Returns dict(base=numpy base dict, post=posterior dict, consts=E-step constants
    (oracle prelude), opt=options, T=tau, bs=BaseSet, P=Posterior)."""
    bs = vb.synth_base_set(N, K, Sb, d, covmode, seed=1000 + seed, device="cpu",
                           exprmt1=exprmt1, ragged=ragged, face=face)
    v0 = max(5.0, d + 1.0)
    if face:  # demo/vbdemo_face.m:49-61 hyperparameters (m0 defaults to [256, 192])
        opt_over = dict(dict(W0=0.001, v0=10.0), **opt_over)
        v0 = opt_over.pop("v0")
    opt = vb.default_options(K, S, d, tau=tau, Nv=Nv, covmode=covmode, v0=v0, **opt_over)
    rb, rg, om = vb.baseem_draws(bs, K, S, seed=77 + seed)
    P = vb.baseem_init(bs, opt, rb, rg, om)
    if perturb:
        rng = np.random.default_rng(500 + seed)
        P.epsilon = P.epsilon * rng.uniform(0.2, 1.8, P.epsilon.shape)
        P.eta = P.eta * rng.uniform(0.2, 1.8, P.eta.shape)
        P.lam = P.lam * rng.uniform(0.5, 1.5, P.lam.shape)
        P.v = P.v + rng.uniform(0.0, 3.0, P.v.shape)
        sc = rng.uniform(0.7, 1.3, P.v.shape)
        P.W = P.W * (sc[..., None, None] if covmode == 1 else sc[..., None])
        P.m = P.m + rng.normal(0.0, 8.0 if face else 0.3, P.m.shape)
        P.alpha = P.alpha * rng.uniform(0.5, 1.5, P.alpha.shape)
    base = bs.numpy()
    post = post_dict(P)
    consts = vo.prelude(post, covmode)
    return dict(base=base, post=post, consts=consts, opt=opt, T=tau, bs=bs, P=P)


# shapes exercised by the parity tests: (name, N, K, S, Sb, d, covmode, T, ragged)
SHAPES = [
    ("full_small", 5, 3, 3, 3, 2, 1, 6, False),
    ("diag_small", 5, 3, 3, 3, 2, 0, 6, False),
    ("T1", 4, 2, 3, 3, 2, 1, 1, False),
    ("T2", 4, 2, 3, 3, 2, 1, 2, False),
    ("S1", 4, 3, 1, 3, 2, 1, 5, False),
    ("Sb1", 4, 3, 3, 1, 2, 1, 5, False),
    ("ragged_full", 9, 3, 4, 4, 3, 1, 7, True),
    ("ragged_diag", 9, 3, 4, 4, 3, 0, 7, True),
    ("SbgtS", 4, 2, 2, 5, 2, 1, 4, False),
    ("odd", 5, 5, 5, 5, 5, 1, 9, False),
    ("d1", 4, 2, 3, 3, 1, 0, 5, False),
    ("C2like", 6, 4, 3, 2, 2, 1, 50, False),
    ("C3like", 6, 8, 5, 5, 2, 0, 10, False),
    ("C4like", 3, 16, 8, 8, 8, 1, 10, False),
    ("C5like", 1, 32, 12, 12, 16, 1, 10, False),
    ("S16", 2, 3, 16, 16, 4, 1, 6, False),
    ("d16diag", 2, 3, 6, 6, 16, 0, 6, False),
    # S = 8, T = 10: the MFMA kernels (fb_bwd4_kernel, fb_list4_kernel); padded base
    # states (SB < 8, ragged) and gate lists that end inside a 4-pair quad
    ("S8_ragged", 9, 5, 8, 6, 3, 1, 10, True),
    ("S8_quads", 37, 4, 8, 8, 2, 0, 10, False),
    # S = 12: the MFMA backward pass on 3 x 3 blocks (fb_bwd12_kernel); SB < 12 pads
    # whole and partial column blocks, a quad ending past the last base
    ("S12_ragged", 9, 5, 12, 9, 3, 1, 10, True),
    ("S12_quads", 37, 4, 12, 12, 2, 0, 10, False),
    ("S12_sb5", 7, 3, 12, 5, 2, 1, 6, False),
    # outside the column-split kernel's limits (S <= 16, SB <= S, d <= 16): generic kernel
    ("d20", 3, 2, 3, 3, 20, 1, 5, False),
    ("S20", 2, 2, 20, 20, 2, 1, 4, False),
    ("T50_SbgtS", 3, 3, 2, 6, 2, 0, 50, True),
]


def make_reduced(K=3, S=3, d=2, covmode=1, seed=0, zero_transition=False) -> dict:
    """Point-estimate reduced HMMs for the VHEM sibling (hem_hmm_bwd_fwd_mex.c):
    Dirichlet rows for A and prior, means in [0, 5]^d, SPD covariances
    (L L'/d + 0.5 I) or diagonal U[0.5, 1.5].  zero_transition sets A[0][0][-1]
    (renormalised) and prior[0][-1] to 0, so log(A) and log(prior) hold -inf."""
    rng = np.random.default_rng(4000 + seed)
    A = rng.dirichlet(np.ones(S), size=(K, S))
    prior = rng.dirichlet(np.ones(S), size=K)
    if zero_transition and S > 1:
        A[0, 0, -1] = 0.0
        A[0, 0] /= A[0, 0].sum()
        prior[0, -1] = 0.0
        prior[0] /= prior[0].sum()
    centres = rng.uniform(0.0, 5.0, (K, S, d))
    if covmode == 1:
        L = rng.normal(size=(K, S, d, d))
        covars = np.einsum("ksab,kscb->ksac", L, L) / d + 0.5 * np.eye(d)
    else:
        covars = rng.uniform(0.5, 1.5, (K, S, d))
    return dict(A=A, prior=prior, centres=centres, covars=covars)

