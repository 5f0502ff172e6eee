"""The clustering API around the device E-step (callers of the hot path).

* :func:`vbhem_h3m_cluster` -- src/vbhem/vbhem_h3m_cluster.m:103-402: input
  HMMs -> remove empty states (:116-134, vbhmm_remove_empty with thresh 1e-3)
  -> ``hmms_to_h3m_hem`` (:237) -> for a vector of K, one run per K and the best
  of LL + gammaln(K+1) (:261-309); for a vector of S, likewise with
  gammaln(S+1) (:313-354); a single (K, S) runs :func:`vbhem_h3m_c`.
* :func:`vbhem_h3m_c` -- vbhem_h3m_c.m:28-76, 167-170: ``trials`` EM runs
  (the reference's ``parfor``) as ONE batched launch per iteration
  (em.vbhem_h3m_c_trials), the best bound wins; with ``learn_hyps`` the
  unique trials (uniqueLL, :79-89) are re-optimised by the L-BFGS
  hyperparameter learner (hyp.vbhem_h3m_c_hyp, :94-137).
* :func:`unique_ll` -- src/util/uniqueLL.m; :func:`form_groups` --
  form_outputH3M.m:50-60 (label, groups, group_size).

Initialisation (opt['initmode']): 'baseem' (the default here; vbhemhmm_init.m:58-100)
with its draws from a numpy generator seeded by seed + trial (vbhem_h3m_c.m:32-38
seeds MATLAB's twister the same way), 'wtkmeans' (vbhemhmm_init.m:294-425:
weighted k-means of the base states' means, h3m.wtkmeans_init; MATLAB's kmeans
replaced by a k-means++ stand-in), 'gmmNew' (vbhemhmm_init.m:103-293: the base
Gaussians reduced by hierarchical EM, GMM_MixHierEM.m, h3m.gmmnew_init), or 'auto'
(vbhem_h3m_cluster.m:359-395: each of the three, the best bound wins).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np
import torch
from scipy.special import gammaln

from . import em
from .estep import EStepEngine
from .h3m import (COV_FULL, BaseSet, baseem_draws, baseem_init, default_options, hmms_to_h3m_hem,
                  hmms_to_h3m_hem_device, gmmnew_init, wtkmeans_init, wtkmeans_points)


def unique_ll(LLall: Sequence[float], diffthresh: float) -> List[int]:
    """uniqueLL.m:43-84: indices of the trials whose bound differs from every
    bound kept so far by more than diffthresh (relative)."""
    kept_ll: List[float] = []
    kept: List[int] = []
    for it, my_LL in enumerate(LLall):
        if it == 0:
            new = True
        else:
            pLL = np.abs((np.asarray(kept_ll) - my_LL) / my_LL)
            new = bool(np.all(pLL > diffthresh))   # MATLAB `if` on a vector: all nonzero
        if new:
            kept_ll.append(float(my_LL))
            kept.append(it)
    return kept


def form_groups(label: np.ndarray, K: int):
    """form_outputH3M.m:50-60: 0-based label -> groups (indices per cluster) and
    group_size."""
    label = np.asarray(label).reshape(-1)
    groups = [np.flatnonzero(label == j) for j in range(K)]
    return groups, np.array([g.size for g in groups])


def _device_engine(device):
    dev = torch.device(device)
    return lambda base, K, S, T, trials=1: EStepEngine(base, K, S, T, device=dev, trials=trials)


def vbhem_h3m_c(base: BaseSet, opt: dict, device="cuda", engine_factory=None,
                hyp_learn: Optional[bool] = None) -> dict:
    """vbhem_h3m_c.m for one (K, S): batched trials, best bound (and optional
    hyperparameter learning of the unique trials).  Trials run in launches of at
    most 256 clusters (vbhem_estep_fused_trials' limit).  ``engine_factory(base,
    K_total, S, T, trials)`` builds the E-step engine (default: the device one)."""
    K, S, R = int(opt["K"]), int(opt["S"]), int(opt.get("trials", 100))
    make = engine_factory or _device_engine(device)
    posts = []
    initmode = opt.get("initmode", "baseem")
    if initmode not in ("baseem", "wtkmeans", "gmmNew"):
        raise ValueError(f"initmode {initmode!r}: 'baseem', 'gmmNew' or 'wtkmeans'")
    pts = wtkmeans_points(base, opt.get("initopt_mode", "r0")) if initmode == "wtkmeans" else None
    if initmode == "gmmNew":
        bn = base.numpy()
        ns = bn["nstates"]
        pts = (np.concatenate([bn["centres"][i, :int(ns[i])] for i in range(base.N)]),
               np.concatenate([bn["covars"][i, :int(ns[i])] for i in range(base.N)]))
    for it in range(1, R + 1):
        if initmode == "wtkmeans":  # vbhem_h3m_c.m:52-54: wtseed = seed + trial
            posts.append(wtkmeans_init(base, opt, int(opt["seed"]) + it, pts))
        elif initmode == "gmmNew":  # (the trial's stream: rng(seed + trial), :32-38)
            posts.append(gmmnew_init(base, opt, int(opt["seed"]) + it, pts))
        else:
            rb, rg, om = baseem_draws(base, K, S, seed=int(opt["seed"]) + it)
            posts.append(baseem_init(base, opt, rb, rg, om))
    results, LLs = [], []
    if S <= 16 and base.SB <= S:
        per = max(1, 256 // K)
        for r0 in range(0, R, per):
            chunk = posts[r0:r0 + per]
            eng = make(base, len(chunk) * K, S, opt["tau"], trials=len(chunk))
            tr = em.vbhem_h3m_c_trials(chunk, eng, opt)
            results.extend(tr.results)
            LLs.extend(tr.LLall.tolist())
            del eng
    else:
        # base HMMs with more states than the clusters (or S > 16): the batched-trials
        # launch needs the column-split kernel (Sb <= S), so the trials run one after
        # another through the single-trial fused E-step (generic kernel)
        one = make(base, K, S, opt["tau"], trials=1)
        for P in posts:
            r = em.vbhem_h3m_c_step_fc(P, one, opt)
            results.append(r)
            LLs.append(r.LL)
    LLall = np.array(LLs)
    learn = opt.get("learn_hyps", 0) if hyp_learn is None else hyp_learn
    hyp_info = None
    if learn:
        from . import hyp
        uniq = unique_ll(LLall, 2 * opt["minDiff"] * 10)
        one = make(base, K, S, opt["tau"], trials=1)
        hyp_info = {}
        # vbhem_h3m_c.m:102-105: every bound is invalidated; only the re-optimised
        # unique trials get one back (:157), so only they can be chosen
        LLall = np.full_like(LLall, np.nan)
        for q in uniq:
            h = hyp.vbhem_h3m_c_hyp(base, opt, results[q].post, one)
            results[q] = h["result"]
            LLall[q] = h["result"].LL
            hyp_info[q] = h
    # vbhem_h3m_c.m:163: MATLAB's max skips NaN (all NaN: the first entry)
    best = 0 if np.all(np.isnan(LLall)) else int(np.nanargmax(LLall))
    res = results[best]
    out = dict(result=res, LL=float(LLall[best]), LLall=LLall, best=best, K=K, S=S,
               hyp=hyp_info[best] if hyp_info and best in hyp_info else None)
    if res.label is not None:
        lab = res.label.cpu().numpy()
        out["label"] = lab
        out["groups"], out["group_size"] = form_groups(lab, K)
    return out


def vbhem_h3m_cluster(hmms: list, K, S, opt: Optional[dict] = None, device="cuda",
                      base: Optional[BaseSet] = None, engine_factory=None) -> dict:
    """vbhem_h3m_cluster.m:103-402 (full covariance, use_post = 1; initmode 'auto'
    unless opt says otherwise, as the reference).  ``hmms``: list of VB-HMM dicts (vbhmm_em output) or None;
    ``base``: an already converted h3m_b (skips the conversion)."""
    Ks = [int(k) for k in np.atleast_1d(K)]
    Ss = [int(s) for s in np.atleast_1d(S)]
    opt = dict(opt or {})
    opt.setdefault("initmode", "auto")  # vbhem_h3m_cluster.m:165
    if base is None:
        from .vbhmm_em import vbhmm_remove_empty
        if opt.get("remove_empty", 1):
            hmms = [vbhmm_remove_empty(h, 1e-3) if h is not None else None for h in hmms]
        if opt.get("convert_on_device", 0) and torch.device(device).type == "cuda":
            base = hmms_to_h3m_hem_device(hmms, COV_FULL, True, device)  # csrc/vbhem_h3m.hip
        else:
            base = hmms_to_h3m_hem(hmms, COV_FULL, use_post=True)
    if len(Ks) > 1:
        outs = [vbhem_h3m_cluster(None, k, Ss, dict(opt), device, base, engine_factory) for k in Ks]
        LLk = np.array([o["LL"] for o in outs]) + gammaln(np.array(Ks) + 1.0)
        ind = int(np.argmax(LLk))
        h = dict(outs[ind])
        h.update(model_LL=LLk, model_k=Ks, model_bestK=Ks[ind], model_all=outs)
        return h
    if len(Ss) > 1:
        outs = [vbhem_h3m_cluster(None, Ks[0], s, dict(opt), device, base, engine_factory)
                for s in Ss]
        LLs = np.array([o["LL"] for o in outs]) + gammaln(np.array(Ss) + 1.0)
        ind = int(np.argmax(LLs))
        h = dict(outs[ind])
        h.update(model_LL_S=LLs, model_S=Ss, model_bestS=Ss[ind], model_all_s=outs)
        return h
    o = default_options(Ks[0], Ss[0], base.d, **{k: v for k, v in opt.items()
                                                  if k not in ("K", "S")})
    if o.get("initmode") == "auto":
        # vbhem_h3m_cluster.m:359-395: every initialisation in turn, each with its own
        # initopt.mode (opt['initmodes'] with opt['initopts'], default {'baseem', 'gmmNew',
        # 'wtkmeans'} with {'u', 'r0', 'r0'}), the best bound wins; keep_best_random_trial
        # (default 1, :208) keeps every mode's run as h3m_out_trials (:391-393).  The
        # 'wtkmeans' / 'gmmNew' centres come from a k-means++ stand-in for MATLAB's kmeans,
        # so which mode wins is parity unpinned.
        if "initmodes" in o:
            modes = list(o["initmodes"])
            if "initopts" not in o or len(o["initopts"]) != len(modes):
                raise ValueError("opt['initmodes'] needs opt['initopts'] of the same length "
                                 "(vbhem_h3m_cluster.m:366-368)")
            iopts = list(o["initopts"])
        else:
            modes, iopts = ["baseem", "gmmNew", "wtkmeans"], ["u", "r0", "r0"]
        runs = []
        for m, io in zip(modes, iopts):
            r = vbhem_h3m_c(base, dict(o, initmode=m, initopt_mode=io), device, engine_factory)
            runs.append(dict(r, Initmodes=m))
        ind = int(np.argmax([r["LL"] for r in runs]))
        out = dict(runs[ind])
        out.update(initmode=modes[ind], init_trials_LL=[r["LL"] for r in runs])
        if o.get("keep_best_random_trial", 1):
            out["h3m_out_trials"] = runs
        out["LL_orignal"] = out["LL"]   # (sic, :398)
        return out
    return vbhem_h3m_c(base, o, device, engine_factory)
