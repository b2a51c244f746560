"""Pin the oracle (CPU restatement) against golden vectors produced by the reference itself.

Tolerance: 1e-4 relative to the tensor's max magnitude for forward tensors (both sides are
fp32 torch-CPU; the restatement reorders a few ops), 1e-3 for losses and gradients.
"""
import numpy as np
import pytest
import torch

import oracle
from oracle import reconet_ref as R
from oracle import shapes

import conftest
from conftest import rel_err


def T(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def test_known_answers():
    # gram_matrix(ones(1,2,3,3)) == 0.5 everywhere (RC/utilities.py:93-98)
    g = R.gram_matrix(torch.ones(1, 2, 3, 3))
    assert torch.allclose(g, torch.full_like(g, 0.5))
    # vgg_normalize mutates its argument to x/255 (RC/utilities.py:105)
    x = torch.full((1, 3, 2, 2), 255.0)
    out = R.vgg_normalize_(x)
    assert torch.allclose(x, torch.ones_like(x))
    assert torch.allclose(out[0, :, 0, 0], (1 - torch.tensor(R.IMAGENET_MEAN)) / torch.tensor(R.IMAGENET_STD))


def test_units(golden):
    u = golden("rc_units")
    for tag in ("img", "feat", "wide", "ramp"):
        flo = u.get(f"warp_{tag}_flo")
        x = T(u[f"warp_{tag}_x"])
        flo = T(flo) if flo is not None else torch.zeros(x.shape[0], 2, *x.shape[2:])
        assert rel_err(R.warp(x, flo), u[f"warp_{tag}_out"]) < 1e-5, tag
    # zero flow is not the identity for this warp
    assert np.abs(u["warp_ramp_out"] - u["warp_ramp_x"]).max() > 1.0
    for i in range(3):
        m = R.flow_warp_mask(T(u[f"fwm{i}_f01"]), T(u[f"fwm{i}_f10"]))
        assert np.array_equal(m.numpy(), u[f"fwm{i}_mask"]), i
    assert rel_err(R.gram_matrix(T(u["gram_y"])), u["gram_out"]) < 1e-6
    x = T(u["vggn_x"]).clone()
    out = R.vgg_normalize_(x)
    assert rel_err(out, u["vggn_out"]) < 1e-6 and rel_err(x, u["vggn_x_after"]) < 1e-7


def test_forward(golden):
    f = golden("rc_fwd")
    P = oracle.seeded_params(shapes.reconet(), 1)
    with torch.no_grad():
        for tag in ("a", "ragged"):
            sd1, feat, out = R.reconet_forward(P, T(f[f"reconet_{tag}_x"]))
            assert rel_err(sd1, f[f"reconet_{tag}_sd1"]) < 1e-4
            assert rel_err(feat, f[f"reconet_{tag}_features"]) < 1e-4
            assert rel_err(out, f[f"reconet_{tag}_out"]) < 1e-4
        VP = oracle.seeded_params(shapes.vgg16(), 4)
        outs = R.vgg_forward(VP, T(f["vgg16_x"]), R.VGG16_PLAN)
        for o, name in zip(outs, ("relu1_2", "relu2_2", "relu3_3", "relu4_3")):
            assert rel_err(o, f["vgg16_" + name]) < 1e-4, name


@pytest.mark.parametrize("tag", ["b2", "b1r"])
def test_train_step(golden, tag):
    s = golden("rc_step")
    seeds = s[f"{tag}_seeds"]
    P = oracle.seeded_params(shapes.reconet(), int(seeds[0]), requires_grad=True)
    VP = oracle.seeded_params(shapes.vgg16(), int(seeds[1]))
    grams = R.style_grams(VP, T(s[f"{tag}_style"]))
    L = R.reconet_losses(P, VP, T(s[f"{tag}_img1"]).clone(), T(s[f"{tag}_img2"]).clone(),
                         T(s[f"{tag}_flow"]), T(s[f"{tag}_mask"]), grams)
    for k in ("loss", "CL", "SL", "FTL", "OTL", "RL"):
        assert rel_err(L[k].item(), s[f"{tag}_{k}"]) < 1e-3, k
    L["loss"].backward()
    names = list(s[f"{tag}_names"])
    assert sorted(names) == sorted(P)
    gmax = max(float(s[f"{tag}_gnorm/{n}"]) for n in names)
    state = {}
    grads = {n: P[n].grad for n in names}
    params = {n: P[n].detach().clone() for n in names}
    R.adam_step(params, grads, state)
    for n in names:
        g = P[n].grad
        gn = float(s[f"{tag}_gnorm/{n}"])
        # each tensor: norm within 1e-3 relative (or 1e-4 of the largest gradient norm)
        assert abs(float(g.double().norm()) - gn) <= 1e-3 * gn + 1e-4 * gmax, n
        idx = s[f"{tag}_gidx/{n}"]
        assert np.abs(g.reshape(-1)[idx].numpy() - s[f"{tag}_gval/{n}"]).max() <= 1e-3 * gn + 1e-4 * gmax, n
        # Adam's first step is ~ -lr*sign(g): compare where the gradient is not round-off noise
        # (conv biases feeding InstanceNorm have mathematically zero gradient)
        gh = s[f"{tag}_ghead/{n}"]
        sel = np.abs(gh) > 1e-6 * gmax + 1e-2 * np.abs(gh).max()
        assert np.abs(params[n].reshape(-1)[:64].numpy() - s[f"{tag}_phead/{n}"])[sel].max(initial=0) < 1e-5, n


@pytest.mark.parametrize("term", R.ALL_TERMS)
@pytest.mark.parametrize("tag", ["b2", "b1r"])
def test_train_step_per_term(golden, tag, term):
    """Each train_candy loss term ALONE (the reference's own train() with the other four weight
    constants zeroed, gen_golden.gen_terms): the oracle's term value and its gradient, tensor by
    tensor, at the per-term bar of conftest.term_grad_margins (TERM_REL of the tensor's own exact norm;
    the oracle itself sits ~1e-6 from the exact gradient on these cases)."""
    d = golden("rc_terms")
    seeds = d[f"{tag}_seeds"]
    P = oracle.seeded_params(shapes.reconet(), int(seeds[0]), requires_grad=True)
    VP = oracle.seeded_params(shapes.vgg16(), int(seeds[1]))
    grams = R.style_grams(VP, T(d[f"{tag}_style"]))
    L = R.reconet_losses(P, VP, T(d[f"{tag}_img1"]).clone(), T(d[f"{tag}_img2"]).clone(),
                         T(d[f"{tag}_flow"]), T(d[f"{tag}_mask"]), grams, terms=(term,))
    p = f"{tag}_{term}_"
    assert rel_err(L["loss"].item(), d[p + "term"]) < 1e-5
    assert rel_err(d[p + "term"], d[p + "exact_loss"]) < 1e-5
    L["loss"].backward()
    grads = {n: (v.grad if v.grad is not None else torch.zeros_like(v)).numpy() for n, v in P.items()}
    m = conftest.term_grad_margins(d, p, grads)
    worst = max(m, key=m.get)
    assert m[worst] <= 1.0, (worst, m[worst])


CLONES = {  # tag: (single, input_frame_num, weights, terms) -- the reference script each golden ran
    "coco": (True, 1, dict(R.LOSS_WEIGHTS, BETA=1e10), ("CL", "SL")),        # train_coco2014.py
    "cocor": (True, 1, dict(R.LOSS_WEIGHTS, BETA=1e10), ("CL", "SL")),
    "noftl": (False, 1, dict(R.LOSS_WEIGHTS, BETA=1e10), ("OTL", "CL", "SL", "RL")),  # train_Flow_noFTL.py
    "multi": (False, 4, dict(R.LOSS_WEIGHTS, BETA=1e10), R.ALL_TERMS),        # train_multiple/train_Flow.py
}


def check_grads(s, tag, grads, after):
    """Per-tensor gradient norm / sampled values (1e-3 of the norm + 1e-4 of the largest norm) and
    the post-Adam parameter heads, against the reference's recorded step."""
    names = list(s[f"{tag}_names"])
    assert sorted(names) == sorted(grads)
    gmax = max(float(s[f"{tag}_gnorm/{n}"]) for n in names)
    for n in names:
        g = grads[n].reshape(-1)
        gn = float(s[f"{tag}_gnorm/{n}"])
        assert abs(float(g.double().norm()) - gn) <= 1e-3 * gn + 1e-4 * gmax, n
        idx = s[f"{tag}_gidx/{n}"]
        assert np.abs(g[idx].numpy() - s[f"{tag}_gval/{n}"]).max() <= 1e-3 * gn + 1e-4 * gmax, n
        gh = s[f"{tag}_ghead/{n}"]
        sel = np.abs(gh) > 1e-6 * gmax + 1e-2 * np.abs(gh).max()
        assert np.abs(after[n].reshape(-1)[:64].numpy() - s[f"{tag}_phead/{n}"])[sel].max(initial=0) < 1e-5, n


@pytest.mark.parametrize("tag", sorted(CLONES))
def test_clone_train_steps(golden, tag):
    """train_coco2014 / train_Flow_noFTL / train_multiple/train_Flow: the oracle vs the
    reference's own train() (tests/golden/gen_golden.py gen_clones)."""
    s = golden("rc_clones")
    single, nfr, w, terms = CLONES[tag]
    assert sorted(terms) == sorted(s[f"{tag}_terms"])
    seeds = s[f"{tag}_seeds"]
    P = oracle.seeded_params(shapes.reconet(nfr), int(seeds[0]), requires_grad=True)
    VP = oracle.seeded_params(shapes.vgg16(), int(seeds[1]))
    grams = R.style_grams(VP, T(s[f"{tag}_style"]))
    if single:
        L = R.reconet_single_losses(P, VP, T(s[f"{tag}_img"]).clone(), grams, w)
    else:
        L = R.reconet_losses(P, VP, T(s[f"{tag}_img1"]).clone(), T(s[f"{tag}_img2"]).clone(),
                             T(s[f"{tag}_flow"]), T(s[f"{tag}_mask"]), grams, w, terms=terms)
    assert sorted(k for k in L if k != "loss") == sorted(terms)
    for k in ("loss",) + tuple(terms):
        assert rel_err(L[k].item(), s[f"{tag}_{k}"]) < 1e-3, k
    L["loss"].backward()
    grads = {n: P[n].grad for n in P}
    params = {n: P[n].detach().clone() for n in P}
    R.adam_step(params, grads, {})
    check_grads(s, tag, grads, params)


# ----------------------------------------------------------------------------- AdaAttN
def test_cosine_moments_exact():
    """oracle.adaattn_ref.cosine_moments_exact (the float64 re-associated yardstick for the config-4/5
    attention sizes) equals the materialised attention_moments in float64, ragged shapes included."""
    from oracle import adaattn_ref as A

    g = torch.Generator().manual_seed(3)
    for b, d, dv, (h, w), (hs, ws) in ((2, 16, 8, (6, 10), (5, 7)), (1, 40, 24, (9, 4), (12, 11))):
        Q = torch.randn(b, d, h, w, generator=g, dtype=torch.float64)
        K = torch.randn(b, d, hs, ws, generator=g, dtype=torch.float64)
        V = torch.randn(b, dv, hs, ws, generator=g, dtype=torch.float64) * 2 + 0.5
        M, S = A.attention_moments(Q, K, V)
        Me, Se = A.cosine_moments_exact(Q, K, V)
        assert rel_err(Me, M) < 1e-12 and rel_err(Se, S) < 1e-12


def test_adaattn_units(golden):
    from oracle import adaattn_ref as A

    u = golden("aa_units")
    VP = oracle.seeded_params(shapes.vgg19(), 31)
    with torch.no_grad():
        fx, fs = A.vgg19(VP, T(u["x"])), A.vgg19(VP, T(u["s"]))
        for k in A.FEATS:
            assert rel_err(fx[k], u[f"vgg19_x_{k}"]) < 1e-4, k
        lx, ls = list(fx.values()), list(fs.values())
        for idx in (2, 3, 4):
            assert rel_err(A.feature_down_sample(lx, idx), u[f"fds_x_{idx}"]) < 1e-5
        for i in range(3):
            idx = i + 2
            c1, s1 = A.feature_down_sample(lx, idx), A.feature_down_sample(ls, idx)
            assert rel_err(A.adaattn(None, None, lx[idx], ls[idx], c1, s1), u[f"noconv{i}"]) < 1e-4, i
        P = oracle.seeded_params(shapes.stylizing_network(), 32)
        for i in range(3):
            idx = i + 2
            c1, s1 = A.feature_down_sample(lx, idx), A.feature_down_sample(ls, idx)
            assert rel_err(A.adaattn(P, f"adaattn.{i}", lx[idx], ls[idx], c1, s1), u[f"adaattn{i}"]) < 1e-4, i
        assert rel_err(A.stylize(P, fx, fs), u["stylized"]) < 1e-4
        for k in ("relu2_1", "relu3_1", "relu4_1", "relu5_1"):
            assert rel_err(A.global_stylized_loss(fx[k], fs[k]).item(), u[f"gsl_{k}"]) < 1e-4, k
        for k in ("relu2_1", "relu3_1", "relu4_1"):
            assert rel_err(A.cosine_distance(fx[k], fs[k]), u[f"cosd_{k}"]) < 1e-5, k
            got = A.image_similarity_loss(fx[k], fs[k], fs[k] * 0.5 + 1.0, fx[k]).item()
            assert rel_err(got, u[f"isl_{k}"]) < 1e-4, k


def test_adaattn_train_step(golden):
    from oracle import adaattn_ref as A

    s = golden("aa_step")
    seeds = s["seeds"]
    P = oracle.seeded_params(shapes.stylizing_network(), int(seeds[0]), requires_grad=True)
    VP = oracle.seeded_params(shapes.vgg19(), int(seeds[1]))
    L = A.adaattn_losses(P, VP, T(s["c1"]), T(s["c2"]), T(s["style"]))
    for k in ("loss", "loss_gs", "loss_lf", "loss_is"):
        assert rel_err(L[k].item(), s[k]) < 1e-3, k
    L["loss"].backward()
    names = list(s["names"])
    assert sorted(names) == sorted(P)
    gmax = max(float(s[f"gnorm/{n}"]) for n in names)
    for n in names:
        g = P[n].grad
        gn = float(s[f"gnorm/{n}"])
        assert abs(float(g.double().norm()) - gn) <= 1e-3 * gn + 1e-4 * gmax, n
        idx = s[f"gidx/{n}"]
        assert np.abs(g.reshape(-1)[idx].numpy() - s[f"gval/{n}"]).max() <= 1e-3 * gn + 1e-4 * gmax, n


def test_adaattn_image_step(golden):
    """The oracle's train_image step (softmax attention, no IS term) vs the reference's own
    AA/train_image.py train() (tests/golden/gen_golden.py gen_aa_image)."""
    from oracle import adaattn_ref as A

    s = golden("aa_image_step")
    seeds = s["seeds"]
    P = oracle.seeded_params(shapes.stylizing_network(), int(seeds[0]), requires_grad=True)
    VP = oracle.seeded_params(shapes.vgg19(), int(seeds[1]))
    L = A.adaattn_image_losses(P, VP, T(s["content"]), T(s["style"]))
    for k in ("loss", "loss_gs", "loss_lf"):
        assert rel_err(L[k].item(), s[k]) < 1e-3, k
    L["loss"].backward()
    names = list(s["names"])
    assert sorted(names) == sorted(P)
    gmax = max(float(s[f"gnorm/{n}"]) for n in names)
    for n in names:
        g = P[n].grad
        gn = float(s[f"gnorm/{n}"])
        assert abs(float(g.double().norm()) - gn) <= 1e-3 * gn + 1e-4 * gmax, n
        idx = s[f"gidx/{n}"]
        assert np.abs(g.reshape(-1)[idx].numpy() - s[f"gval/{n}"]).max() <= 1e-3 * gn + 1e-4 * gmax, n


# ----------------------------------------------------------------------------- distillation (SD2)
SD_WEIGHTS = dict(ALPHA=1e5, BETA=1e10, GAMMA=1e-2, LAMBDA_F=1e11, LAMBDA_O=1e7)  # train_Flow_SD2.py:24-29


def sd2_params(seeds, requires_grad=False):
    """Teacher ReCoNetSD1 and student ReCoNetSD2 as train_Flow_SD2.py:42-45 builds them: the student's
    res*_sd blocks come from the teacher checkpoint (load_state_dict(strict=False))."""
    TP = oracle.seeded_params(shapes.reconet_sd1(), int(seeds[0]))
    P = oracle.seeded_params(shapes.reconet_sd2(), int(seeds[1]))
    for k in P:
        if k in TP:
            P[k] = TP[k].clone()
    for v in P.values():
        v.requires_grad_(requires_grad)
    return TP, P


def test_sd2_train_step(golden):
    s = golden("sd_step")
    assert any("train_Flow_SD1.py" in str(n) for n in s["notes"])  # the reference's SD1 trainer cannot load
    seeds = s["sd2_seeds"]
    TP, P = sd2_params(seeds, requires_grad=True)
    VP = oracle.seeded_params(shapes.vgg16(), int(seeds[2]))
    grams = R.style_grams(VP, T(s["sd2_style"]))
    L = R.reconet_losses(P, VP, T(s["sd2_img1"]).clone(), T(s["sd2_img2"]).clone(), T(s["sd2_flow"]),
                         T(s["sd2_mask"]), grams, w=SD_WEIGHTS, forward=R.reconet_sd2_forward,
                         teacher=(TP, R.reconet_sd1_forward, 0, 0))
    for k in ("loss", "CL", "SL", "FTL", "OTL", "RL", "SDL"):
        assert rel_err(L[k].item(), s[f"sd2_{k}"]) < 1e-3, k
    L["loss"].backward()
    names = list(s["sd2_names"])
    gmax = max(float(s[f"sd2_gnorm/{n}"]) for n in names)
    for n in names:
        g = P[n].grad
        gn = float(s[f"sd2_gnorm/{n}"])
        assert abs(float(g.double().norm()) - gn) <= 1e-3 * gn + 1e-4 * gmax, n
