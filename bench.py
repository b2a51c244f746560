"""Benchmark: ReCoNet training frame-pairs/s at 256x512 on MI355X (BASELINE.json metric).

Workload (one "step"): the reference `train_candy` loop body (RC/train_single/train_candy.py:77-152)
on one batch of B synthetic frame pairs per GPU, 3x256x512, precomputed flow + occlusion mask,
full loss (FTL + OTL + content + Gram style + TV) through the Vgg16 loss network, backward and
Adam — config 3 of BASELINE.json.  `--config 2` runs the reference's no-temporal script
(train_coco2014.py: content + Gram style on the 2B single frames of B pairs).  Random-init weights
(no checkpoint download offline), synthetic data already resident in HBM.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one rank per GPU, RCCL all-reduce)

`python bench.py --gpus N` with N > 1 outside torchrun starts the N ranks itself: before any GPU
call it runs `python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1
--master-port P bench.py <same arguments>` as a child process and relays rank 0's JSON line (exit
code = the child's).  Under torchrun, `--gpus` must equal WORLD_SIZE.  `--dry-run` replaces the
training step with a CPU stand-in (gloo gradient all-reduce) to test that launcher on a machine
without GPUs.

Inputs: every step trains on its own synthetic batch, numpy PCG64 seeded 1234 + step on rank 0
([1234 + step, rank] on the others), all generated and staged in HBM before the
timed region.

GEMM arithmetic (`--gemm`, vst.ops.POLICIES): the headline runs `bf16x6` -- every conv / Gram
product on three-way split bf16 MFMAs, per-product error ~2^-24 (fp32-class; the reference's
golden steps pass at the f32 bar under it, tests/test_gpu_parity.py) at 2500/6 = 417 TFLOP/s
peak; `f32` is exact fp32 MFMA (157.3 TFLOP/s).

Prints ONE JSON line (rank 0).  `value` comes from K uninstrumented steps.  `roofline` = the
dominant kernel family (conv_gemm_kernel: conv forward + data-gradient implicit GEMM),
algorithmic FLOPs / HIP-event-timed launch time over a second, instrumented run of the same step
(events on the launching stream around every launch) vs the peak of the arithmetic launched.
`cpu_baseline` = the oracle (CPU restatement of the same step, oracle/reconet_ref.py) on a bounded
sample, rank 0 at N=1; `full_size_parity` = the HIP step vs that oracle step on the same B=1
full-size pair (loss terms and gradients).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "video-style-transfer_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (GPUs of this node); > 1 outside torchrun: bench.py launches them itself")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU stand-in step over gloo (tests the multi-rank launcher and timing without GPUs)")
    ap.add_argument("--steps", type=int, default=150)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--prof-steps", type=int, default=10, help="instrumented steps for the roofline line")
    ap.add_argument("--model", default="reconet", choices=("reconet", "adaattn", "reconet_infer", "dataprep"),
                    help="reconet: BASELINE configs 2/3 (the metric); adaattn: config 4's train_video step")
    ap.add_argument("--batch", type=int, default=None, help="frame pairs per GPU (default 8 reconet, 4 adaattn)")
    ap.add_argument("--height", type=int, default=256)
    ap.add_argument("--width", type=int, default=512)
    ap.add_argument("--config", type=int, default=3, choices=(2, 3))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--replay-input", action="store_true",
                    help="A/B only: replay the first synthetic batch every step instead of one batch per step")
    ap.add_argument("--no-vgg19", action="store_true", help="skip the VGG19 fwd+dgrad north-star sub-benchmark")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="oracle threads (default: os.cpu_count(), capped by OMP_NUM_THREADS = the box's CPU share)")
    ap.add_argument("--cpu-steps", type=int, default=5, help="timed oracle steps (median)")
    ap.add_argument("--cpu-warmup", type=int, default=2)
    ap.add_argument("--gemm", default=os.environ.get("VST_GEMM_POLICY"),
                    help="GEMM arithmetic policy, a name in vst.ops.POLICIES (bf16x6, f32, parity, bf16x3, bf16, "
                         "f16); default bf16x6 (fp32-class split products), f16 for the config-5 AdaAttN shape "
                         "(BASELINE's half-precision path)")
    return ap.parse_args()


def cpu_threads(args):
    """Threads for the oracle: os.cpu_count(), capped by OMP_NUM_THREADS when set (the GPU box
    exports the CPU share of one GPU there; os.cpu_count() reports the whole machine)."""
    if args.cpu_threads:
        return args.cpu_threads
    n = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    return min(n, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else n


# oracle / reference time ratio measured in the build container (tools/ref_ratio.py, same step,
# same host, same threads): relates the on-box oracle number to the reference itself
RATIO_FILE = os.path.join(REPO, "profiles", "r02_oracle_ref_ratio.json")


def oracle_ref_ratio(kind):
    if not os.path.exists(RATIO_FILE):
        return None
    return json.load(open(RATIO_FILE)).get(kind)


def _median_rate(one, warmup, steps):
    for i in range(warmup):
        t0 = time.perf_counter()
        one()
        print(f"[bench] cpu warm-up step {i}: {time.perf_counter() - t0:.2f} s", file=sys.stderr, flush=True)
    ts = []
    for i in range(steps):
        t0 = time.perf_counter()
        one()
        ts.append(time.perf_counter() - t0)
        print(f"[bench] cpu step {i}: {ts[-1]:.2f} s", file=sys.stderr, flush=True)
    ts.sort()
    return ts[len(ts) // 2], ts


def cpu_baseline(args):
    """Oracle (CPU restatement of the reference step) on a bounded sample: B=1 pair at full size,
    `cpu_warmup` + `cpu_steps` steps, median.  Also returns the first step's loss terms and
    gradients (before its Adam update) for the full-size parity check."""
    import oracle
    from oracle import reconet_ref as R
    from oracle import shapes
    from vst.synthetic import frame_pair_batch, style_image

    nt = cpu_threads(args)
    torch.set_num_threads(nt)
    H, W = args.height, args.width
    P = oracle.seeded_params(shapes.reconet(), 1, requires_grad=True)
    VP = oracle.seeded_params(shapes.vgg16(), 2)
    grams = R.style_grams(VP, style_image(3, H, W))
    img1, img2, flow, mask = frame_pair_batch(1234, 1, H, W, mask_fn=R.flow_warp_mask)
    state = {}
    first = {"P0": {k: p.detach().clone() for k, p in P.items()}, "VP": VP,
             "inputs": (img1, img2, flow, mask, style_image(3, H, W))}
    w = dict(R.LOSS_WEIGHTS, BETA=1e10) if args.config == 2 else R.LOSS_WEIGHTS

    def one():
        if args.config == 2:  # train_coco2014 on the pair's 2 frames as single images
            L = R.reconet_single_losses(P, VP, torch.cat([img1, img2]), grams, w)
        else:
            L = R.reconet_losses(P, VP, img1.clone(), img2.clone(), flow, mask, grams)
        for p in P.values():
            p.grad = None
        L["loss"].backward()
        if "terms" not in first:
            first.update(terms={k: float(v) for k, v in L.items()}, grads={k: p.grad.clone() for k, p in P.items()})
        with torch.no_grad():
            R.adam_step({k: p for k, p in P.items()}, {k: p.grad for k, p in P.items()}, state)

    med, ts = _median_rate(one, args.cpu_warmup, args.cpu_steps)
    # the same first step in float64 (exact up to float64 rounding): the yardstick the full-size gate
    # holds both the HIP step and the fp32 oracle step to
    P64 = {k: v.double().requires_grad_(True) for k, v in first["P0"].items()}
    VP64 = {k: v.double() for k, v in VP.items()}
    g64 = R.style_grams(VP64, style_image(3, H, W).double())
    if args.config == 2:
        L = R.reconet_single_losses(P64, VP64, torch.cat([img1, img2]).double(), g64, w)
    else:
        L = R.reconet_losses(P64, VP64, img1.double(), img2.double(), flow.double(), mask.double(), g64)
    L["loss"].backward()
    first["terms64"] = {k: float(v.detach()) for k, v in L.items()}
    first["grads64"] = {k: (p.grad if p.grad is not None else torch.zeros_like(p)).detach() for k, p in P64.items()}
    res = {"value": 1.0 / med, "unit": "frame-pairs/s", "cores": nt, "kind": "port",
           "os_cpu_count": os.cpu_count(),
           "sample": f"median of {args.cpu_steps} timed steps (+{args.cpu_warmup} warm-up) of a B=1 synthetic "
                     f"3x{H}x{W} frame pair, config {args.config}, oracle/reconet_ref.py on torch-CPU fp32, "
                     f"{nt} threads", "step_s": ts,
           "oracle_to_reference_time_ratio": oracle_ref_ratio("reconet")}
    return res, first


def cpu_baseline_adaattn(args):
    """Oracle AdaAttN train_video step (oracle/adaattn_ref.py) on B=1 triple at full size."""
    import oracle
    from oracle import adaattn_ref as A
    from oracle import shapes
    from vst.synthetic import content_style_batch

    nt = cpu_threads(args)
    torch.set_num_threads(nt)
    H, W = args.height, args.width
    P = oracle.seeded_params(shapes.stylizing_network(), 1, requires_grad=True)
    VP = oracle.seeded_params(shapes.vgg19(), 2)
    c1, c2, s = content_style_batch(99, 1, H, W)
    from oracle import reconet_ref as R

    state = {}
    first = {"P0": {k: p.detach().clone() for k, p in P.items()}, "VP": VP, "inputs": (c1, c2, s)}

    def one():
        L = A.adaattn_losses(P, VP, c1, c2, s)
        for p in P.values():
            p.grad = None
        L["loss"].backward()
        if "terms" not in first:
            first.update(terms={k: float(v) for k, v in L.items()}, grads={k: p.grad.clone() for k, p in P.items()})
        with torch.no_grad():
            R.adam_step(P, {k: p.grad for k, p in P.items()}, state, lr=1e-4)

    steps, warm = max(1, args.cpu_steps // 2), min(1, args.cpu_warmup)
    med, ts = _median_rate(one, warm, steps)
    return {"value": 1.0 / med, "unit": "frame-pairs/s", "cores": nt, "kind": "port", "os_cpu_count": os.cpu_count(),
            "sample": f"median of {steps} timed step(s) (+{warm} warm-up) of a B=1 synthetic 3x{H}x{W} (content1, "
                      f"content2, style) triple, oracle/adaattn_ref.py on torch-CPU fp32, {nt} threads",
            "step_s": ts, "oracle_to_reference_time_ratio": oracle_ref_ratio("adaattn")}, first


# config-5 policy (single bf16 products): the bar tests/test_gpu_adaattn.py states for it
BF16_BAR = {"loss_rel": 2e-2, "gnorm_rel_of_gn_plus_0.1gmax": 5e-2, "sampled_cosine_min": 0.99}


def adaattn_level_parity(model, vgg, c, s, ref_form=True):
    """Each AdaAttN level's two attention moments M (AA/network.py:208) and S = sqrt(clamp(E2 - M^2))
    (:209-213) from the HIP path (the current GEMM policy, linear form) vs the float64 exact value
    (oracle.adaattn_ref.cosine_moments_exact) on the SAME Q, K, V (the HIP 1x1 convs of the HIP VGG19
    features), so only the attention arithmetic is measured; `ref_form`: the reference's own
    materialised fp32 form (oracle.adaattn_ref.attention_moments) on the same Q, K, V beside it.
    S is read through the product's output kernel: out = S * cn + M with cn = 0 gives M, with
    cn = 2^20 gives S = (out - M) / 2^20 (exact scaling; the add rounds at 2^-24 of S * 2^20)."""
    from oracle import adaattn_ref as A
    from vst import ops
    from vst.adaattn.attention import COSINE, adaattn, instance_norm_plain
    from vst.adaattn.utilities import feature_down_sample

    def rel(x, e):
        x, e = x.double().cpu(), e.double().cpu()
        return {"max": float((x - e).abs().max() / e.abs().max()), "norm": float((x - e).norm() / e.norm())}

    out = []
    with torch.no_grad():
        fc, fs = list(vgg(c).values()), list(vgg(s).values())
        for i in range(3):
            idx, mod = i + 2, model.adaattn[i]
            with ops.gemm_scope("stylizer"), ops.gemm_scope("attn"):  # (the policy scope AdaAttN's own convs run in)
                Q = ops.conv2d(instance_norm_plain(feature_down_sample(fc, idx)), mod.f.weight, mod.f.bias)
                K = ops.conv2d(instance_norm_plain(feature_down_sample(fs, idx)), mod.g.weight, mod.g.bias)
                V = ops.conv2d(fs[idx], mod.h.weight, mod.h.bias)
                shp = (Q.shape[0], V.shape[1]) + tuple(Q.shape[2:])
                M = adaattn(Q, K, V, torch.zeros(shp, device=Q.device), COSINE)
                S = (adaattn(Q, K, V, torch.full(shp, 2.0 ** 20, device=Q.device), COSINE) - M) * 2.0 ** -20
            Qc, Kc, Vc = Q.cpu(), K.cpu(), V.cpu()
            Me, Se = A.cosine_moments_exact(Qc, Kc, Vc)
            e = {"level": FEATS_AA[idx], "Nc": Q.shape[2] * Q.shape[3], "Ns": K.shape[2] * K.shape[3],
                 "d": Q.shape[1], "dv": V.shape[1], "hip": {"M": rel(M, Me), "S": rel(S, Se)}}
            if ref_form:
                Mr, Sr = A.attention_moments(Qc, Kc, Vc)
                e["reference_form_fp32"] = {"M": rel(Mr, Me), "S": rel(Sr, Se)}
                del Mr, Sr
            out.append(e)
    return out


FEATS_AA = ("relu1_1", "relu2_1", "relu3_1", "relu4_1", "relu5_1")


def full_size_parity_adaattn(args, dev, first):
    """The HIP train_video step (current GEMM policy) vs the oracle step on the SAME B=1 full-size
    triple and initial weights (cpu_baseline_adaattn's first step): loss terms, per-tensor gradient
    norms, sampled-gradient cosine, and each attention level's M / S vs float64."""
    from vst import ops
    from vst.adaattn.network import StylizingNetwork
    from vst.adaattn.train import AdaAttNTrainer
    from vst.adaattn.vgg19 import VGG19

    c1, c2, s = first["inputs"]
    model = StylizingNetwork("cosine")
    model.load_state_dict(first["P0"])
    vgg = VGG19()
    vgg.load_state_dict(first["VP"])
    model, vgg = model.to(dev), vgg.to(dev)
    tr = AdaAttNTrainer(model, vgg, activation="cosine")
    tr.flat.zero_grad()
    out = tr.losses(torch.stack([c1, c2, s]).to(dev))
    unscale = tr.backward(out["loss"])
    torch.cuda.synchronize()
    ref = first["terms"]
    terms = {k: abs(float(out[k]) - ref[k]) / abs(ref[k]) for k in ref}
    g = {n: p.grad.detach().double().cpu().reshape(-1) * unscale for n, p in model.named_parameters()}
    gr = {n: first["grads"][n].double().reshape(-1) for n in g}
    gmax = max(float(v.norm()) for v in gr.values())
    gerr = {n: abs(float(g[n].norm()) - float(gr[n].norm())) / (float(gr[n].norm()) + 0.1 * gmax) for n in g}
    margin = max((abs(float(g[n].norm()) - float(gr[n].norm())) / (1e-3 * float(gr[n].norm()) + 1e-4 * gmax), n)
                 for n in g)
    a = torch.cat([g[n] / (gr[n].norm() + 1e-30) for n in g])
    b = torch.cat([gr[n] / (gr[n].norm() + 1e-30) for n in g])
    cos = float(a @ b / (a.norm() * b.norm()))
    flat = float(torch.cat([g[n] - gr[n] for n in g]).norm() / torch.cat(list(gr.values())).norm())
    levels = adaattn_level_parity(model, vgg, c1.to(dev), s.to(dev))
    single_bf16 = ops.policy_modes() in (["bf16"], ["f16"])
    res = {"workload": f"B=1 3x{args.height}x{args.width} (content1, content2, style) triple, same seeded weights/inputs",
           "gemm_policy": args.gemm, "loss_rel_err": terms,
           "grad_norm_margin_worst": {"tensor": margin[1], "margin": margin[0],
                                      "bar": "1e-3 norm + 1e-4 largest norm (fp32-class golden bar)"},
           "grad_norm_err_worst": {"tensor": max(gerr, key=gerr.get), "err": max(gerr.values()),
                                   "bar": "|norm - ref| / (ref + 0.1 largest)"},
           "grad_cosine_whole": cos, "grad_rel_err_flat": flat, "attention_levels": levels}
    if single_bf16:
        res["bar"] = BF16_BAR
        res["pass"] = bool(max(terms.values()) <= BF16_BAR["loss_rel"]
                           and max(gerr.values()) <= BF16_BAR["gnorm_rel_of_gn_plus_0.1gmax"]
                           and cos >= BF16_BAR["sampled_cosine_min"])
    else:
        res["bar"] = {"loss_rel": 1e-3, "grad_norm_margin": 1.0}
        res["pass"] = bool(max(terms.values()) < 1e-3 and margin[0] <= 1.0)
    return res


def pmc_traffic(model, family=("conv_halo_kernel", "conv_gemm_kernel")):
    """HBM bytes per launch of the roofline kernel family from the committed PMC summary of the same
    workload (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, tools/pmc_traffic.py; counters cannot
    be read from inside the timed run): the launch-weighted mean over the family's kernels.  None if
    no summary is committed."""
    import glob

    files = sorted(glob.glob(os.path.join(REPO, "profiles", f"r*_traffic_{model}.json")))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    fams = [d["families"][f] for f in ((family,) if isinstance(family, str) else family) if f in d["families"]]
    if not fams:
        return None, None
    launches = sum(f.get("launches", 1) for f in fams)
    total = sum(f["bytes_per_launch"] * f.get("launches", 1) for f in fams)
    return total / launches, os.path.relpath(files[-1], REPO) + " (" + d["method"] + ")"


def vgg19_subbench(dev, reps=3, B=8, H=256, W=512):
    """SURVEY.md §8(d) north-star sub-metric: VGG19 features[0:21] (to relu4_1) forward + input
    gradient on B=8x3x256x512, random-init frozen weights.  Returns conv-kernel TFLOP/s (HIP events
    around every conv_gemm launch) and the wall-clock rate of the whole fwd+dgrad pass."""
    from vst import kprof
    from vst.adaattn.vgg19 import VGG19
    from vst.reconet.network import run_vgg_slice

    vgg = VGG19().to(dev)
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(B, 3, H, W, device=dev, generator=g).requires_grad_(True)
    cfg = [(3, 64, H, W), (64, 64, H, W), (64, 128, H // 2, W // 2), (128, 128, H // 2, W // 2),
           (128, 256, H // 4, W // 4), (256, 256, H // 4, W // 4), (256, 256, H // 4, W // 4),
           (256, 256, H // 4, W // 4), (256, 512, H // 8, W // 8)]
    fwd_flops = sum(2.0 * B * co * h * w * ci * 9 for ci, co, h, w in cfg)

    def one():
        f = x
        for s in range(1, 5):
            f = run_vgg_slice(getattr(vgg, f"slice{s}"), f)
        f.backward(torch.ones_like(f))
        x.grad = None

    one()
    torch.cuda.synchronize()
    timer = kprof.KernelTimer()
    t0 = time.perf_counter()
    with timer:
        for _ in range(reps):
            one()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps
    ks = timer.summary()
    peak = ks["peak_tflops"]
    return {"workload": f"VGG19 features[0:21] (relu4_1) fwd + input grad, B={B}x3x{H}x{W}",
            "algo_gflop": 2 * fwd_flops / 1e9, "conv_tflops": ks["tflops"], "peak_tflops": peak,
            "conv_frac": ks["tflops"] / peak, "wall_tflops": 2 * fwd_flops / wall / 1e12,
            "wall_frac": 2 * fwd_flops / wall / 1e12 / peak, "ms": wall * 1e3,
            "wall_frac_of_fp32_mfma_peak": 2 * fwd_flops / wall / 1e12 / FP32_MFMA_PEAK_TFLOPS,
            "target_frac": 0.60}


def build_reconet(args, dev, rank):
    from vst import ops
    from vst.reconet import network as N
    from vst.reconet.train import ReCoNetTrainer
    from vst.synthetic import frame_pair_parts, style_image

    model = N.ReCoNet().to(dev)
    vgg = N.Vgg16().to(dev)
    B, H, W = args.batch, args.height, args.width
    style = style_image(7, H, W).to(dev)
    script = "train_coco2014" if args.config == 2 else "train_candy"
    trainer = ReCoNetTrainer.for_script(script, model, vgg, style)

    def stage(parts):
        # (staged before the timed region; the frame stack and the motion product on the host, so the
        # device runs only the library's kernels)
        img1, img2, f01, f10, motion = parts
        frames = torch.stack([img1, img2]).contiguous().to(dev)
        if trainer.single:  # config 2: the 2B frames of the B pairs as single images
            return (frames.reshape(2 * B, 3, H, W),)
        # occlusion mask on the device (RC/utilities.py:60-90, batched) x the motion stand-in
        occ = ops.flow_warp_mask(f01.contiguous().to(dev), f10.contiguous().to(dev))
        mask = (occ.cpu() * motion).contiguous().to(dev)
        return frames, f10.contiguous().to(dev), mask

    batches = per_step_batches(args, rank, lambda seed: frame_pair_parts(seed, B, H, W), stage)
    return cycle_steps(trainer.step, batches)


def full_size_parity(args, dev, first):
    """The HIP step (current GEMM policy) vs the oracle step on the SAME B=1 full-size frame pair
    and initial weights (cpu_baseline's first step, before its Adam update): relative error of
    every loss term, of the flattened gradient, and the worst per-tensor gradient-norm error."""
    from vst.reconet import network as N
    from vst.reconet.train import ReCoNetTrainer

    img1, img2, flow, mask, style = first["inputs"]
    model = N.ReCoNet()
    model.load_state_dict(first["P0"])
    vgg = N.Vgg16()
    vgg.load_state_dict(first["VP"])
    script = "train_coco2014" if args.config == 2 else "train_candy"
    tr = ReCoNetTrainer.for_script(script, model.to(dev), vgg.to(dev), style.to(dev))
    if tr.single:
        out = tr.losses(torch.cat([img1, img2]).to(dev))
    else:
        out = tr.losses(torch.stack([img1, img2]).to(dev), flow.to(dev), mask.to(dev))
    tr.flat.zero_grad()
    out["loss"].backward()
    torch.cuda.synchronize()
    ref, ref64 = first["terms"], first["terms64"]
    terms = {k: abs(float(out[k]) - ref[k]) / abs(ref[k]) for k in ref}
    terms64 = {k: abs(float(out[k]) - ref64[k]) / abs(ref64[k]) for k in ref64}
    g = {n: p.grad.detach().double().cpu().reshape(-1) for n, p in model.named_parameters()}
    gr = {n: first["grads"][n].double().reshape(-1) for n in g}
    ge = {n: first["grads64"][n].reshape(-1) for n in g}

    def flat_err(a, b):
        return float(torch.cat([a[n] - b[n] for n in g]).norm() / torch.cat([b[n] for n in g]).norm())

    flat, flat64, oracle64 = flat_err(g, gr), flat_err(g, ge), flat_err(gr, ge)
    gmax = max(float(v.norm()) for v in gr.values())
    # per tensor: |norm - ref norm| / (1e-3 ref norm + 1e-4 largest ref norm) -- the golden-step bar of
    # tests/test_gpu_parity.py, <= 1 passes
    margin = max((abs(float(g[n].norm()) - float(gr[n].norm())) / (1e-3 * float(gr[n].norm()) + 1e-4 * gmax), n)
                 for n in g)
    tol = 1e-3
    # flat gradient gate: the HIP step's distance from the float64 step within 2x the fp32 oracle's own
    # distance from it (single gradient elements are conditioned by ReLU / InstanceNorm decisions, so
    # the bar is what fp32 itself achieves on this input, not a fixed number)
    flat_bar = 2.0 * oracle64
    return {"workload": f"B=1 3x{args.height}x{args.width} frame pair, config {args.config}, same seeded weights/inputs",
            "tolerance": tol, "loss_rel_err": terms, "loss_rel_err_vs_float64": terms64,
            "grad_norm_margin_worst": {"tensor": margin[1], "margin": margin[0]},
            "grad_rel_err_flat": flat,
            "grad_rel_err_flat_vs_float64": flat64,
            "oracle_fp32_grad_rel_err_flat_vs_float64": oracle64,
            "grad_flat_gate": {"bar": flat_bar, "rule": "HIP vs float64 <= 2 x (fp32 oracle vs float64)",
                               "pass": bool(flat64 <= flat_bar)},
            "pass": bool(max(terms.values()) < tol and margin[0] <= 1.0 and flat64 <= flat_bar)}


def build_adaattn(args, dev, rank):
    from vst.adaattn.network import StylizingNetwork
    from vst.adaattn.train import AdaAttNTrainer
    from vst.adaattn.vgg19 import VGG19
    from vst.synthetic import content_style_batch

    model = StylizingNetwork("cosine").to(dev)
    vgg = VGG19().to(dev)
    trainer = AdaAttNTrainer(model, vgg, activation="cosine")
    B, H, W = args.batch, args.height, args.width
    batches = per_step_batches(args, rank, lambda seed: content_style_batch(seed, B, H, W),
                               lambda cs: (torch.stack(cs).contiguous().to(dev),))
    return cycle_steps(trainer.step, batches)


def per_step_batches(args, rank, draw, stage):
    """One synthetic batch per step (warm-up, timed and instrumented steps), seeded
    vst.reconet.dist.step_seed(step, rank) = 1234 + step on rank 0; drawn on host
    threads (numpy releases the GIL in its fills), staged in HBM before the timed region."""
    from concurrent.futures import ThreadPoolExecutor

    from vst.reconet.dist import step_seed

    n = 1 if args.replay_input else args.warmup + args.steps + args.prof_steps
    ranks_here = max(int(os.environ.get("LOCAL_WORLD_SIZE", "1")), 1)
    workers = max(1, min(8, (os.cpu_count() or 1) // ranks_here))
    t0 = time.perf_counter()
    out = []
    with ThreadPoolExecutor(workers) as ex:
        for c0 in range(0, n, 2 * workers):  # bounded host memory: 2 x workers batches in flight
            for parts in ex.map(lambda i: draw(step_seed(i, rank)), range(c0, min(n, c0 + 2 * workers))):
                out.append(stage(parts))
    print(f"[bench] {n} per-step batches staged in {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    return out


def cycle_steps(step_fn, batches):
    """step() trains on batch i of the per-step list at its i-th call (wrapping after the last)."""
    it = {"i": 0}

    def step():
        b = batches[it["i"] % len(batches)]
        it["i"] += 1
        return step_fn(*b)

    step.trainer = getattr(step_fn, "__self__", None)
    return step


def build_reconet_infer(args, dev, rank):
    """ReCoNet video inference (RC/utilities.py:179-235) on B frames per
    step: uint8 BGR frames resident in HBM -> frames_to_tensor -> ReCoNet forward (no_grad) ->
    clamp + BGR + uint8 (tensor_to_frames).  Frames are independent (input_frame_num=1)."""
    from vst import ops
    from vst.reconet import network as N
    from vst.reconet.dist import shard_seed
    from vst.synthetic import video_frames

    model = N.ReCoNet().to(dev).eval()
    frames = torch.from_numpy(video_frames(shard_seed(1234, rank), args.batch, args.height, args.width)).to(dev)
    out = torch.empty_like(frames)

    def step():
        with torch.no_grad():
            x = ops.frames_to_tensor(frames)
            *_, y = model(x)
            ops.tensor_to_frames(y, frames=out)
        return {}

    return step


def cpu_baseline_infer(args):
    """Oracle ReCoNet inference (oracle/reconet_ref.py) on one 360x640 frame."""
    import oracle
    from oracle import reconet_ref as R
    from oracle import shapes
    from vst.synthetic import video_frames

    nt = cpu_threads(args)
    torch.set_num_threads(nt)
    P = oracle.seeded_params(shapes.reconet(), 1)
    frames = video_frames(5, 1 + args.cpu_steps, args.height, args.width)
    R.inference(R.reconet_forward, P, frames[:1], 1)  # warm-up
    t0 = time.perf_counter()
    R.inference(R.reconet_forward, P, frames[1:], 1)
    dt = (time.perf_counter() - t0) / args.cpu_steps
    return {"value": 1.0 / dt, "unit": "frames/s", "cores": nt, "kind": "port",
            "sample": f"{args.cpu_steps} frames (+1 warm-up) of synthetic 3x{args.height}x{args.width} video, "
                      f"oracle/reconet_ref.py inference on torch-CPU fp32, {nt} threads"}


def run_dataprep(args, dev, rank, world):
    """the device half of FlyingThings3D / Monkaa `__getitem__`
    (RC/datasets.py:114-146) for B frame pairs per step, inputs resident in HBM at the dataset's
    source size (960x540 PNG frames / PGM motion boundaries as uint8, PFM flows as raw float bits)
    -> 640x360 training items (vst.reconet.datasets.prepare_staged's kernels)."""
    import numpy as np

    from vst import ops
    from vst.reconet.dist import shard_seed

    B, (Hs, Ws), (Ho, Wo) = args.batch, (540, 960), (360, 640)
    rng = np.random.default_rng(shard_seed(1234, rank))
    frames = torch.from_numpy(rng.integers(0, 256, (2 * B, Hs, Ws, 3), dtype=np.uint8)).to(dev)
    motion = torch.from_numpy(np.where(rng.random((B, Hs, Ws)) < 0.05, 255, 0).astype(np.uint8)).to(dev)
    # SURVEY.md §8(d) synthetic flow: a 2x(H/16)x(W/16) U(-8, 8) px field bilinearly upsampled
    # (PFM layout: H x W x 3, third channel zero, rows bottom-up -- the flip is irrelevant to the data)
    coarse = torch.from_numpy(rng.uniform(-8, 8, (2 * B, 2, Hs // 16, Ws // 16)).astype(np.float32))
    fine = torch.nn.functional.interpolate(coarse, size=(Hs, Ws), mode="bilinear", align_corners=False)
    raw = torch.cat([fine, torch.zeros(2 * B, 1, Hs, Ws)], dim=1).permute(0, 2, 3, 1).contiguous().numpy()
    flows = torch.from_numpy(raw.astype("<f4").view(np.int32)).to(dev)
    img = torch.empty((2 * B, 3, Ho, Wo), device=dev)
    fl = torch.empty((2 * B, 2, Ho, Wo), device=dev)

    def resize_frames():
        ops.pil_resize_to_tensor255(frames, (Wo, Ho), out=img)

    def step():
        resize_frames()
        ops.flow_prep(flows, False, (Wo, Ho), out=fl)
        mask = ops.flow_warp_mask(fl[:B], fl[B:])
        ops.apply_motion_mask(mask, motion)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    elapsed = float(elapsed.item())
    # dominant kernel: the Pillow-exact frame resize, timed with HIP events on its own stream
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record(st)
    for _ in range(reps):
        resize_frames()
    e1.record(st)
    torch.cuda.synchronize()
    us = 1e3 * e0.elapsed_time(e1) / reps
    algo = 2 * B * (Hs * Ws * 3 + 3 * Ho * Wo * 4)  # uint8 HWC frames in, fp32 planes out
    if rank != 0:
        return None
    traffic, traffic_src = pmc_traffic("dataprep", "pil_resize_kernel<3, 5, 5>")
    result = {
        "metric": "frame-pair items/sec, FlyingThings3D __getitem__ device half (960x540 -> 640x360)",
        "value": B * world * args.steps / elapsed, "unit": "items/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8/f32",
        "data": "synthetic (numpy PCG64 uint8 frames, 5% motion-boundary pixels, smooth flows: "
                "U(-8,8) px at 1/16 resolution, bilinearly upsampled, SURVEY.md §8(d))",
        "config": {"workload": f"dataprep: B={B} items/GPU, frames+motion 960x540 uint8, PFM flows 960x540x3 "
                               f"-> img1/img2 3x360x640, flow 2x360x640, mask 360x640", "global_batch": B * world,
                   "parallelism": f"dp{world}"},
        "roofline": {"bound": "hbm", "kernel": "pil_resize_kernel<3, 5, 5> (frames, mode 0)",
                     "achieved": algo / us / 1e3, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": algo / us / 1e3 / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     "algo_bytes_per_launch": algo, "avg_launch_us": us},
    }
    if world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline_dataprep(args)
    print(json.dumps(result), flush=True)
    return result


def cpu_baseline_dataprep(args):
    """The oracle's item pipeline (Pillow resize + torch-CPU flow resize + oracle mask) per item."""
    import numpy as np

    from oracle import dataprep_ref as D
    from oracle import reconet_ref as R

    nt = cpu_threads(args)
    torch.set_num_threads(nt)
    rng = np.random.default_rng(7)
    n = max(args.cpu_steps, 2)
    items = [([rng.integers(0, 256, (540, 960, 3), dtype=np.uint8) for _ in range(2)],
              rng.uniform(-20, 20, (540, 960, 3)).astype(np.float32),
              rng.uniform(-20, 20, (540, 960, 3)).astype(np.float32),
              np.where(rng.random((540, 960)) < 0.05, 255, 0).astype(np.uint8)) for _ in range(n + 1)]
    D.getitem(*items[0], (640, 360), R.flow_warp_mask)
    t0 = time.perf_counter()
    for it in items[1:]:
        D.getitem(*it, (640, 360), R.flow_warp_mask)
    dt = (time.perf_counter() - t0) / n
    return {"value": 1.0 / dt, "unit": "items/s", "cores": nt, "kind": "port",
            "sample": f"{n} items (+1 warm-up), decoded inputs, oracle/dataprep_ref.getitem (numpy Pillow "
                      f"restatement + torch-CPU bilinear + oracle flow_warp_mask), {nt} threads"}


def default_policy(args):
    if args.gemm:
        return args.gemm
    if args.model == "adaattn" and (args.height, args.width) == (512, 1024):
        # config 5: BASELINE's fp16 MFMA path (convolutions on fp16 products under a dynamic loss
        # scale; the attention modules, the image-similarity products and the loss network's forward
        # over the stylised frames on bf16x3).  Single-bf16
        # products fail the policy's own bar at this size
        return "f16"
    return "bf16x6"


def arithmetic_label(ops, ks):
    """dtype string: fp32 operands/accumulation + the product arithmetic actually launched."""
    names = sorted({ops.gemm_mode_name(m) for m in ks["by_mode"]}) or ops.policy_modes()
    desc = {"f32": "f32 MFMA", "bf16x6": "bf16x6 split MFMA (~2^-24/product)", "bf16x3": "bf16x3 split MFMA (~2^-16)",
            "bf16": "bf16 MFMA (~2^-8)", "f16": f"fp16 MFMA (~2^-11, dynamic loss scale from {ops.loss_scale():g})"}
    base = names[0] if names in (["bf16"], ["f16"]) else "f32"
    return f"{base} ({' + '.join(desc[n] for n in names)})"


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize()


def timed(step, steps, world, dev, mark=False):
    _sync(dev)
    if world > 1:
        dist.barrier()
    if mark:  # rocprofv3 marker dispatch: the counter passes select the dispatches after it
        from vst._lib import lib, stream

        lib.vst_marker(stream())
    _sync(dev)
    t0 = time.perf_counter()
    out = None
    for _ in range(steps):
        out = step()
    _sync(dev)
    if world > 1:
        dist.barrier()
    elapsed = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    return float(elapsed.item()), out


def launch_ranks(args):
    """`--gpus N` (N > 1) without a torchrun environment: run the N ranks as a child
    torch.distributed.run (one process per GPU, RCCL over xGMI), relay rank 0's JSON line, return the
    child's exit code.  Called before anything touches the GPU (this process never initialises HIP)."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    print(f"[bench] launching {args.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, text=True)
    for line in proc.stdout:  # rank 0 prints the JSON line; anything else goes to stderr
        (sys.stdout if line.lstrip().startswith("{") else sys.stderr).write(line)
        sys.stdout.flush()
    return proc.wait()


def dry_run(args, world, rank):
    """CPU stand-in for the training step (no GPU): a fixed matmul chain per frame pair plus the
    step's one gradient all-reduce (15.05 MB, ReCoNet's flat gradient) over gloo, timed exactly as
    the real line (barrier, max over ranks).  Exercises the launcher, the rank environment and the
    line's aggregation; its `value` says nothing about MI355X."""
    dev = torch.device("cpu")
    B = args.batch
    g = torch.Generator().manual_seed(rank)
    a = torch.randn(256, 256, generator=g)
    grad = torch.zeros(3763011)

    def step():
        for _ in range(B):
            a.copy_(torch.tanh(a @ a) * 0.5)
        if world > 1:
            dist.all_reduce(grad)
        return {}

    for _ in range(args.warmup):
        step()
    elapsed, _ = timed(step, args.steps, world, dev)
    if rank != 0:
        return None
    value = B * world * args.steps / elapsed
    result = {"metric": "dry run (CPU stand-in step; launcher test)", "value": value, "unit": "frame-pairs/s",
              "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
              "ms_per_step": 1e3 * elapsed / args.steps, "higher_is_better": True, "scaling": "weak",
              "vs_baseline": None, "dtype": "f32", "data": "none (dry run)",
              "config": {"workload": "dry run", "global_batch": B * world, "parallelism": f"dp{world}"},
              "elapsed_s": elapsed}
    print(json.dumps(result), flush=True)
    return result


def main():
    args = parse()
    if args.batch is None:
        args.batch = {"reconet": 8, "adaattn": 4, "reconet_infer": 16, "dataprep": 8}[args.model]
    if args.model == "reconet_infer" and (args.height, args.width) == (256, 512):
        args.height, args.width = 360, 640  # RC/utilities.py:121 (inference frame size)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if (args.gpus or 1) > 1:
            sys.exit(launch_ranks(args))  # N ranks as a child torchrun; nothing here touched the GPU
        world = 1
    else:
        world = int(env_world)
        if args.gpus is not None and args.gpus != world:
            print(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr, flush=True)
            sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        if world > 1:
            dist.init_process_group("gloo")
        res = dry_run(args, world, rank)
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return res
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from vst import kprof, ops

    if args.model == "dataprep":
        return run_dataprep(args, dev, rank, world)
    args.gemm = default_policy(args)
    ops.use_policy(args.gemm)
    torch.manual_seed(0)  # identical random-init replicas on every rank (the trainers also broadcast rank 0's)
    B, H, W = args.batch, args.height, args.width
    step = {"reconet": build_reconet, "adaattn": build_adaattn, "reconet_infer": build_reconet_infer}[args.model](
        args, dev, rank)

    for _ in range(args.warmup):
        step()
    # headline: K uninstrumented steps
    elapsed, out = timed(step, args.steps, world, dev, mark=True)
    # roofline: a second run of the same step with HIP events around every conv_gemm launch, the side
    # streams off so that each launch has the chip to itself: its duration is
    # the kernel's, not shared with a concurrent weight-gradient GEMM (the timed region above runs them
    # on; tools/gpu_r04_close.sh profiles with the same switches so the rocprofv3 averages compare)
    timer = kprof.KernelTimer()
    side = (ops.WGRAD_SIDE, ops.CONTENT_SIDE)
    ops.WGRAD_SIDE = ops.CONTENT_SIDE = False
    try:
        with timer:
            prof_elapsed, _ = timed(step, args.prof_steps, world, dev)
    finally:
        ops.WGRAD_SIDE, ops.CONTENT_SIDE = side
    ks = timer.summary()
    loss = float(out["loss"].item()) if "loss" in out else None

    result = None
    if rank == 0:
        value = B * world * args.steps / elapsed
        achieved = ks["tflops"]
        c5 = args.model == "adaattn" and (H, W) == (512, 1024)
        # the counter summary of this very workload and policy (the strict-f32 line has its own)
        tag = "adaattn_c5" if c5 else (f"{args.model}_f32" if args.gemm == "f32" else args.model)
        traffic, traffic_src = pmc_traffic(tag)
        if args.model == "reconet":
            metric = "training frame-pairs/sec at 256\u00d7512, ReCoNet+VGG19 loss, 1/2/4/8 GPUs"
            workload = (f"config{args.config}: ReCoNet {'train_candy step, full loss incl. FTL/OTL warp' if args.config == 3 else 'train_coco2014 step (content + Gram style, no temporal) on the 2B frames'}"
                        f" (Vgg16 loss net), B={B} frame pairs/GPU, 3x{H}x{W}")
            data = "synthetic (numpy PCG64 frames U[0,255), smooth flow, flow_warp_mask x Bernoulli(0.9)); random-init weights"
        elif args.model == "reconet_infer":
            metric = f"inference frames/sec at {H}\u00d7{W}, ReCoNet (Inference.__iter__ per-frame chain)"
            workload = (f"ReCoNet inference: B={B} uint8 BGR frames/GPU resident in HBM -> fp32 planes -> ReCoNet "
                        f"forward -> clamp/BGR/uint8, 3x{H}x{W}")
            data = "synthetic (numpy PCG64 noise strip panned 3 px/frame); random-init weights"
        else:
            metric = f"training frame-pairs/sec at {H}\u00d7{W}, AdaAttN train_video step (VGG19 encoder/loss)"
            shape = "config5 shape" if (H, W, B) == (512, 1024, 8) else "config4 shape"
            workload = (f"{shape}: AdaAttN train_video step (cosine attention, gs+lf+is losses), "
                        f"B={B} (content1, content2, style) triples/GPU, 3x{H}x{W}")
            data = "synthetic (numpy PCG64 images U[0,255)); random-init weights"
        result = {
            "metric": metric,
            "value": value,
            "unit": "frames/s" if args.model == "reconet_infer" else "frame-pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": arithmetic_label(ops, ks),
            "gemm_policy": {"name": args.gemm, "base": ops.POLICIES[args.gemm][0],
                            "overrides": ops.POLICIES[args.gemm][1]},
            "data": data,
            "config": {"workload": workload,
                       "global_batch": B * world, "height": H, "width": W, "parallelism": f"dp{world}"},
            "frames_per_s": 2 * value,
            "loss_last_step": loss,
            "roofline": {"bound": "mfma", "kernel": "conv fwd + dgrad implicit GEMM (conv_halo_kernel: 3x3 stride-1 "
                                                           "convs; conv_gemm_kernel: the rest), all tile variants",
                         "achieved": achieved, "peak": ks["peak_tflops"], "unit": "TFLOP/s",
                         "frac": achieved / ks["peak_tflops"], "traffic": traffic,
                         "peak_note": "algorithmic fp32-operand TFLOP/s vs the MFMA peak of the arithmetic launched "
                                      "(f32 157.3, bf16x6 2500/6, bf16x3 2500/3, bf16 2500; a mix: flops / "
                                      "sum(flops_i / peak_i))",
                         "frac_of_fp32_mfma_peak": achieved / FP32_MFMA_PEAK_TFLOPS,
                         "by_mode": {ops.gemm_mode_name(m): v for m, v in ks["by_mode"].items()},
                         "traffic_source": traffic_src,
                         "algo_bytes_per_launch": ks["bytes"] / max(ks["launches"], 1),
                         "launches": ks["launches"], "avg_launch_us": ks["avg_us"],
                         "algo_gflop_per_launch": ks["flops"] / max(ks["launches"], 1) / 1e9,
                         "measured_over": f"{args.prof_steps} instrumented steps after the timed region, side streams off "
                                          f"({1e3 * prof_elapsed / max(args.prof_steps, 1):.2f} ms/step instrumented)",
                         "share_of_step": ks["total_ms"] / max(1e3 * prof_elapsed, 1e-9)},
        }
        trainer = getattr(step, "trainer", None)
        if getattr(trainer, "scaler", None) is not None:
            # the fp16 dynamic loss scale after the run: skipped (overflowed) steps did no update
            result["loss_scaler"] = trainer.scaler.state_dict()
        wg = timer.summary("wgrad")
        if wg["launches"]:
            result["roofline"]["wgrad_kernel"] = {"achieved": wg["tflops"], "peak": wg["peak_tflops"],
                                                  "frac": wg["tflops"] / wg["peak_tflops"],
                                                  "share_of_step": wg["total_ms"] / max(1e3 * prof_elapsed, 1e-9)}
        if args.model == "reconet_infer":
            del result["frames_per_s"]
        if world == 1 and not args.no_vgg19 and args.model != "reconet_infer":
            # SURVEY §8(d) sub-metric (>= 60 % of the MFMA roofline of the chosen precision) under exact
            # fp32 MFMA, and under the step's own policy for comparison
            ops.use_policy("f32")
            result["north_star_vgg19"] = vgg19_subbench(dev)
            result["north_star_vgg19"]["gemm_policy"] = "f32"
            if args.gemm != "f32":
                ops.use_policy(args.gemm)
                v = vgg19_subbench(dev)
                result["north_star_vgg19"]["under_step_policy"] = {
                    "gemm_policy": args.gemm, **{k: v[k] for k in ("conv_tflops", "peak_tflops", "conv_frac",
                                                                    "wall_tflops", "wall_frac", "ms")}}
            ops.use_policy(args.gemm)
        if world == 1 and not args.no_cpu_baseline:
            if args.model == "reconet":
                result["cpu_baseline"], first = cpu_baseline(args)
                result["full_size_parity"] = full_size_parity(args, dev, first)
            elif args.model == "adaattn":
                result["cpu_baseline"], first = cpu_baseline_adaattn(args)
                result["full_size_parity"] = full_size_parity_adaattn(args, dev, first)
            else:
                result["cpu_baseline"] = cpu_baseline_infer(args)
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return result


if __name__ == "__main__":
    main()
