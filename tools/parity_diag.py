#!/usr/bin/env python3
"""Parity diagnostics at the benchmarked geometries: the HIP path's errors against the fp32 oracle and
the fp64 oracle, beside the fp32 oracle's own error against fp64 (the noise floor a tolerance has to
clear).  Prints one JSON line per case (PARITY_DIAG {...}).

  c4     ProbUNetTrainer architecture, 256x256, batch 32 (the bench geometry): loss, reconstruction,
         gradients; then 16 injected prior samples through Fcomb (sample_many) + per-class Dice.
  fullw  the same architecture at 64x48, batch 2.
  c5     UNet(3, 3, [64..1024]) at 512x512x3, batch 2, torch.autocast(bfloat16) vs the oracle's
         autocast arithmetic (Bf16Conv3x3).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "probabilistic-multiplanar-unet_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
from helpers import grad_err, max_abs  # noqa: E402

dev = torch.device("cuda")
torch.set_num_threads(min(16, os.cpu_count() or 1))
FULL = (64, 128, 256, 512, 1024)


def emit(name, d):
    print("PARITY_DIAG " + json.dumps({"case": name, **d}), flush=True)


def _inject(dist, eps, method):
    def draw(sample_shape=torch.Size()):
        v = dist.base_dist.loc + dist.base_dist.scale * eps
        return v if method == "rsample" else v.detach()
    setattr(dist, method, draw)


def probunet_case(name, N, H, W, seed, samples):
    from model import ProbabilisticUnet
    from oracle.probunet_ref import fcomb_forward, probunet_param_keys, probunet_train_step
    from oracle.unet_ref import trainer_dice
    from pmu_hip.metrics import dice_counts, dice_from_counts
    torch.manual_seed(0)
    net = ProbabilisticUnet(1, 3, list(FULL), latent_dim=6, no_convs_fcomb=4, beta=10.0).to(dev).train()
    sd = {k: v.detach().cpu().clone() for k, v in net.state_dict().items()}
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(N, 1, H, W, generator=g)
    segm = torch.randint(0, 3, (N, 1, H, W), generator=g).float()
    eps = torch.randn(N, 6, generator=g)
    eps_prior = torch.randn(samples, N, 6, generator=g)
    t0 = time.time()
    res32, g32 = probunet_train_step(dict(sd), x, segm, eps, 5, 6, 3, 4, 10.0)
    t1 = time.time()
    print(f"{name}: fp32 oracle {t1 - t0:.1f} s", flush=True)
    sd64 = {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in sd.items()}
    res64, g64 = probunet_train_step(sd64, x.double(), segm.double(), eps.double(), 5, 6, 3, 4, 10.0)
    t2 = time.time()
    print(f"{name}: fp64 oracle {t2 - t1:.1f} s", flush=True)
    net.forward(x.to(dev), segm.to(dev), training=True)
    _inject(net.posterior_latent_space, eps.to(dev), "rsample")
    elbo = net.elbo(segm.to(dev))
    (-elbo).backward()
    torch.cuda.synchronize()
    named = dict(net.named_parameters())
    keys = [k for k in probunet_param_keys(sd) if not k.startswith("unet.outc")]
    got = {k: named[k].grad for k in keys}
    out = {"N": N, "H": H, "W": W, "oracle32_s": round(t1 - t0, 1), "oracle64_s": round(t2 - t1, 1),
           "loss": float(-elbo), "loss_ref32": float(res32["loss"]), "loss_ref64": float(res64["loss"]),
           "rec_absmax": float(res64["rec"].abs().max()),
           "rec_err32": max_abs(net.reconstruction, res32["rec"]),
           "rec_err64": max_abs(net.reconstruction, res64["rec"]),
           "rec_floor": max_abs(res32["rec"], res64["rec"]),
           "feat_err32": max_abs(net.unet_features, res32["feat"]),
           "grad_err32": grad_err(got, {k: g32[k] for k in keys}),
           "grad_err64": grad_err(got, {k: g64[k] for k in keys}),
           "grad_floor": grad_err({k: g32[k] for k in keys}, {k: g64[k] for k in keys})}
    out["loss_rel32"] = abs(out["loss"] - out["loss_ref32"]) / abs(out["loss_ref32"])
    out["loss_rel64"] = abs(out["loss"] - out["loss_ref64"]) / abs(out["loss_ref64"])
    out["loss_floor"] = abs(out["loss_ref32"] - out["loss_ref64"]) / abs(out["loss_ref64"])
    # evaluation sweep: injected prior samples through the fused Fcomb + per-class Dice counts
    with torch.no_grad():
        d = net.prior_latent_space
        ep = eps_prior.to(dev)
        d.sample = lambda shape=torch.Size(): (d.base_dist.loc + d.base_dist.scale * ep)
        ys = net.sample_many(samples)
        torch.cuda.synchronize()
        mu_p, ls_p = res32["mu_p"], res32["ls_p"]
        zs = mu_p[None] + torch.exp(ls_p)[None] * eps_prior
        sdf = {k: v for k, v in sd.items() if k.startswith("fcomb.")}
        feat = res32["feat"]
        serr, dgap = 0.0, 0.0
        for s in range(samples):
            yr = fcomb_forward(sdf, feat, zs[s], 4)
            serr = max(serr, max_abs(ys[s], yr))
            dh = dice_from_counts(dice_counts(ys[s], segm.to(dev), 3)[None])[0, 1:].tolist()
            dr = trainer_dice(yr, segm, 3)
            dgap = max(dgap, max(abs(a - b) for a, b in zip(dh, dr)))
            agree = float((ys[s].argmax(0 if ys[s].dim() == 3 else 1).cpu() == yr.argmax(1)).float().mean())
        out.update({"samples": samples, "sample_err32": serr, "sample_dice_gap": dgap,
                    "last_sample_label_agreement": agree,
                    "prior_mu_err": max_abs(d.base_dist.loc, mu_p)})
    emit(name, out)


def c5_case(N, S):
    from model import UNet
    from oracle.unet_ref import trainer_dice, unet_forward, unet_loss, unet_param_keys
    torch.manual_seed(0)
    net = UNet(3, 3, list(FULL))
    sd = {k: v.clone() for k, v in net.state_dict().items()}
    g = torch.Generator().manual_seed(2)
    x = torch.rand(N, 3, S, S, generator=g)
    tgt = torch.randint(0, 3, (N, 1, S, S), generator=g)
    keys = unet_param_keys(sd)

    def oracle(dt):
        sdd = {k: (v.to(dt) if v.is_floating_point() else v.clone()) for k, v in sd.items()}
        params = {k: sdd[k].clone().requires_grad_(True) for k in keys}
        work = dict(sdd)
        work.update(params)
        o = unet_forward(work, x.to(dt), 5, 3, bf16=True)
        lo = unet_loss(o, tgt, 3)
        lo.backward()
        return o.detach(), float(lo), {k: params[k].grad for k in keys}, work

    t0 = time.time()
    ref, lref, gref, work = oracle(torch.float64)
    print(f"c5: fp64 oracle {time.time() - t0:.1f} s", flush=True)
    o32, l32, g32, _ = oracle(torch.float32)
    t1 = time.time()
    net = net.to(dev).train()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = net(x.to(dev))
    loss = unet_loss(out, tgt.to(dev), 3)
    loss.backward()
    torch.cuda.synchronize()
    named = dict(net.named_parameters())

    def rel(a, b):
        a, b = a.detach().double().cpu(), b.detach().double().cpu()
        return float((a - b).abs().max() / b.abs().max())
    lab, lab_ref, lab32 = out.argmax(1).cpu(), ref.argmax(1), o32.argmax(1)
    dh, dr, d32 = trainer_dice(out.detach().cpu(), tgt, 3), trainer_dice(ref, tgt, 3), trainer_dice(o32, tgt, 3)
    rs = {}
    for k, v in net.state_dict().items():
        if k.endswith("running_mean") or k.endswith("running_var"):
            rs[k] = float((v.double().cpu() - work[k]).abs().max())
    emit("c5_bf16", {"N": N, "S": S, "oracle_s": round(t1 - t0, 1),
                     "out_rel64": rel(out, ref), "out_floor": rel(o32, ref),
                     "loss_rel64": abs(float(loss) - lref) / abs(lref), "loss_floor": abs(l32 - lref) / abs(lref),
                     "grad_err64": grad_err({k: named[k].grad for k in keys}, gref),
                     "grad_floor": grad_err(g32, gref),
                     "label_agreement64": float((lab == lab_ref).float().mean()),
                     "label_agreement_floor": float((lab32 == lab_ref).float().mean()),
                     "dice_gap64": max(abs(a - b) for a, b in zip(dh, dr)),
                     "dice_floor": max(abs(a - b) for a, b in zip(d32, dr)),
                     "running_stat_err_max": max(rs.values())})


if __name__ == "__main__":
    which = sys.argv[1:] or ["fullw", "c5", "c4"]
    for w in which:
        if w == "fullw":
            probunet_case("fullw", 2, 64, 48, 7, 16)
        elif w == "c4":
            probunet_case("c4", int(os.environ.get("C4N", "32")), 256, 256, 11, 16)
        elif w == "c5":
            c5_case(2, 512)
