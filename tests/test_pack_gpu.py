"""GPU check of the Winograd weight packs (pmu_conv3x3_pack_wino2h / _pack_wino4) against an fp64
restatement of the packed layout, on ragged channel counts (partial co blocks and chunks are zero).

Layouts (csrc/conv3x3_wino2h.hip, csrc/conv3x3_wino4.hip): [co block][chunk of 8][ci in chunk][co in
block][components]; F(2x2): 64 co per block, components 4a+b of G g G^T as four 16-B units, unit q of row
r = ci_in_chunk * 64 + co_in_block stored at q ^ ((r >> 2) & 3) (round 6's unpadded swizzle); F(4x4): 32 co
per block, the 36 components 6a+b of G g G^T in component-half order (upos).  The input-gradient
packs transform w[co][ci] rotated by 180 degrees, with ci as the output channel.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

G2 = torch.tensor([[1, 0, 0], [0.5, 0.5, 0.5], [0.5, -0.5, 0.5], [0, 0, 1]], dtype=torch.float64)
G4 = torch.tensor([[1 / 4, 0, 0], [-1 / 6, -1 / 6, -1 / 6], [-1 / 6, 1 / 6, -1 / 6], [1 / 24, 1 / 12, 1 / 6],
                   [1 / 24, -1 / 12, 1 / 6], [0, 0, 1]], dtype=torch.float64)


def _upos(half, cl):
    return 16 * half + cl if cl < 16 else 32 + 2 * half + (cl - 16)


def _expected(w, dgrad, G, CO, ncp, order=None, swz=False):
    w = w.double().cpu()
    if dgrad:  # filters indexed [out = ci][reduction = co], rotated
        w = w.flip(2, 3).transpose(0, 1)
    nout, kc = w.shape[:2]
    u = torch.einsum("ia,jkab,lb->jkil", G, w, G).reshape(nout, kc, -1)  # [out][k][comp]
    nco, nch = -(-nout // CO), -(-kc // 8)
    ncomp = u.shape[2]
    full = torch.zeros(nco * CO, nch * 8, ncomp, dtype=torch.float64)
    full[:nout, :kc] = u
    if order is not None:
        full = full[:, :, order]
    if ncp > ncomp:
        full = torch.cat([full, torch.zeros(full.shape[0], full.shape[1], ncp - ncomp, dtype=torch.float64)], 2)
    # [co block][col][chunk][kl][comp] -> [co block][chunk][kl][col][comp]
    out = full.reshape(nco, CO, nch, 8, ncp).permute(0, 2, 3, 1, 4).contiguous()
    if swz:  # position p of row r holds unit p ^ ((r >> 2) & 3) (XOR is its own inverse)
        out = out.reshape(nco, nch, 8 * CO, ncp // 4, 4)
        r = torch.arange(8 * CO)
        src = torch.arange(ncp // 4)[None, :] ^ ((r[:, None] >> 2) & 3)
        out = torch.gather(out, 3, src[None, None, :, :, None].expand(nco, nch, -1, -1, 4))
    return out.reshape(-1)


_ORDER4 = [0] * 36
for _c in range(36):
    _ORDER4[_upos(_c // 18, _c % 18)] = _c


@pytest.mark.parametrize("Cout,Cin", [(64, 64), (40, 24), (128, 72), (96, 8)])
@pytest.mark.parametrize("dgrad", [False, True])
def test_pack_wino2h(dev, Cout, Cin, dgrad):
    from pmu_hip import _lib as L
    g = torch.Generator().manual_seed(Cout * 7 + Cin)
    w = torch.randn(Cout, Cin, 3, 3, generator=g).to(dev)
    n = L.lib().pmu_conv3x3_packed_size_wino2h(Cout, Cin, int(dgrad)) // 4
    wp = torch.full((n,), float("nan"), device=dev)
    L.call("pmu_conv3x3_pack_wino2h", w.data_ptr(), Cout, Cin, int(dgrad), wp.data_ptr(), L.stream())
    torch.cuda.synchronize()
    ref = _expected(w, dgrad, G2, 64, 16, swz=True)
    assert ref.numel() == n
    assert float((wp.double().cpu() - ref).abs().max()) <= 1e-6 * float(ref.abs().max())


@pytest.mark.parametrize("Cout,Cin", [(64, 64), (40, 24), (96, 72), (32, 8)])
@pytest.mark.parametrize("dgrad", [False, True])
def test_pack_wino4(dev, Cout, Cin, dgrad):
    from pmu_hip import _lib as L
    g = torch.Generator().manual_seed(Cout * 5 + Cin)
    w = torch.randn(Cout, Cin, 3, 3, generator=g).to(dev)
    n = L.lib().pmu_conv3x3_packed_size_wino4(Cout, Cin, int(dgrad)) // 4
    wp = torch.full((n,), float("nan"), device=dev)
    L.call("pmu_conv3x3_pack_wino4", w.data_ptr(), Cout, Cin, int(dgrad), wp.data_ptr(), L.stream())
    torch.cuda.synchronize()
    ref = _expected(w, dgrad, G4, 32, 36, order=_ORDER4)
    assert ref.numel() == n
    # U is computed in double and rounded once: equal to the fp64 restatement rounded to fp32
    assert float((wp.double().cpu() - ref.float().double()).abs().max()) <= 1e-7 * float(ref.abs().max())


def test_packs_cached_and_batch_repacked_after_fused_sgd(dev):
    """Packed weights are reused until their tensor changes; FusedSGD re-packs every cached layout of
    the parameters it updated in one batched launch per (layout, direction) — the result equals a
    fresh single-tensor pack of the new weights bit for bit, and a second forward/backward launches no
    pack kernel (ragged widths exercise every batched layout's tail blocks)."""
    from model import UNet
    from pmu_hip import engine
    from pmu_hip.optim import FusedSGD
    torch.manual_seed(0)
    net = UNet(1, 1, [32, 64, 128]).to(dev).train()
    opt = FusedSGD(net.parameters(), lr=0.05, momentum=0.9, clip=0.1)
    x = torch.rand(2, 1, 64, 48, device=dev)
    t = (torch.rand(2, 1, 64, 48, device=dev) > 0.5).float()
    calls = []
    orig = dict(engine._LAYOUTS)
    try:
        for k, (fn, multi) in orig.items():
            engine._LAYOUTS[k] = ((lambda f, kk: (lambda w, d: (calls.append(kk), f(w, d))[1]))(fn, k), multi)
        for step in range(3):
            opt.zero_grad()
            torch.nn.functional.binary_cross_entropy(net(x), t).backward()
            opt.step()
            if step == 0:
                first = len(calls)
        assert first > 0 and len(calls) == first, (first, len(calls))   # steps 1, 2: all packs from the cache
    finally:
        engine._LAYOUTS.update(orig)
    torch.cuda.synchronize()
    n = 0
    for (wid, layout, dgrad), e in list(engine._PACKS.items()):
        w = e.w()
        if w is None or not any(w is p for p in net.parameters()):
            continue
        assert e.epoch == w._pmu_epoch and e.ver == w._version
        fresh = orig[layout][0](w, dgrad)
        torch.cuda.synchronize()
        assert torch.equal(e.t, fresh), (layout, dgrad, tuple(w.shape))
        n += 1
    assert n >= 8


def test_channel_mismatch_refused(dev):
    """A filter list that does not double per level makes the decoder's concatenation (skip + up)
    differ from the DoubleConv's in_channels: torch's conv raises there, and so does the engine —
    before any kernel indexes the weight by the operand's channel count."""
    from model import UNet
    net = UNet(1, 1, [32, 48, 64]).to(dev).train()
    with pytest.raises(RuntimeError, match="channels"):
        net(torch.rand(2, 1, 64, 48, device=dev))
    torch.cuda.synchronize()


def test_data_write_needs_invalidate_packs(dev):
    """The pack cache keys on storage, torch's version counter and the FusedSGD epoch.  A write through
    ``.data`` (a custom optimizer, a raw broadcast) bumps none of them: the forward then still runs the
    old packs — the documented hazard — and after invalidate_packs() it runs the new weights, equal to a
    fresh model built from them.  load_state_dict writes in place through the version counter, so a
    checkpoint load is seen without help."""
    from model import UNet
    from pmu_hip import engine
    torch.manual_seed(0)
    net = UNet(1, 1, [32, 64]).to(dev).eval()
    x = torch.rand(2, 1, 64, 48, device=dev)
    sd0 = {k: v.clone() for k, v in net.state_dict().items()}
    # the packed weights (every 3x3 conv but the first layer, which reads its weight raw, and the
    # transposed conv); the head reads its weight raw too
    packed = [k for k, v in sd0.items() if v.dim() == 4 and k not in ("inc.double_conv.0.weight", "outc.conv.weight")]
    assert len(packed) >= 5
    with torch.no_grad():
        y0 = net(x).clone()
        new = {k: (v * 0.5 if k in packed else v) for k, v in sd0.items()}
        for k, p in net.named_parameters():
            p.data.copy_(new[k])                          # not seen by the cache
        y_stale = net(x).clone()
        engine.invalidate_packs()
        y1 = net(x).clone()
        torch.manual_seed(0)
        ref = UNet(1, 1, [32, 64]).to(dev).eval()
        ref.load_state_dict(new)
        y_ref = ref(x).clone()
        net.load_state_dict(sd0)                          # a checkpoint load: in place, version counter bumped
        y2 = net(x)
    torch.cuda.synchronize()
    assert torch.equal(y_stale, y0)                       # the hazard: old packs
    assert not torch.equal(y1, y0)
    assert torch.equal(y1, y_ref)                         # after invalidate_packs(): the new weights
    assert torch.equal(y2, y0)                            # the load is seen without invalidate_packs()


def _expected_dma(w, dgrad):
    """The LDS-DMA bf16 layout (csrc/conv3x3_bf16_dma.hip, pack_dma_body): wp[jb][ch][tap][u][e], unit u =
    2 co + (q XOR bit 3 of co) holding B[tap][k = 16 ch + 8 q + e][j = BN jb + co]; forward B[tap][ci][co] =
    w[co][ci][tap], input gradient B[tap][co][ci] = w[co][ci][8 - tap]; zero padded, bf16 RNE."""
    wf = w.float().cpu().reshape(w.shape[0], w.shape[1], 9)
    B = wf.flip(2).permute(2, 0, 1) if dgrad else wf.permute(2, 1, 0)   # [tap][k][j]
    KC, NOUT = B.shape[1], B.shape[2]
    BN = 64 if (NOUT <= 64 or -(-KC // 16) * 16 <= 128) else 128
    njb, nch = -(-NOUT // BN), -(-KC // 16)
    full = torch.zeros(9, nch * 16, njb * BN)
    full[:, :KC, :NOUT] = B
    X = full.reshape(9, nch, 2, 8, njb, BN).permute(4, 1, 0, 5, 2, 3)   # [jb][ch][tap][co][q][e]
    u = torch.arange(2 * BN)
    co = u >> 1
    q = (u & 1) ^ ((co >> 3) & 1)
    return X[:, :, :, co, q, :].contiguous().reshape(-1).to(torch.bfloat16)


@pytest.mark.parametrize("Cout,Cin", [(64, 64), (40, 24), (128, 72), (256, 160), (96, 8)])
@pytest.mark.parametrize("dgrad", [False, True])
def test_pack_dma(dev, Cout, Cin, dgrad):
    """The bf16 LDS-DMA pack (one 16-B unit per thread) equals the layout restatement bit for bit."""
    from pmu_hip import _lib as L
    g = torch.Generator().manual_seed(Cout * 3 + Cin + int(dgrad))
    w = torch.randn(Cout, Cin, 3, 3, generator=g).to(dev)
    n = L.lib().pmu_conv3x3_packed_size_dma(Cout, Cin, int(dgrad)) // 2
    wp = torch.full((n,), -1, dtype=torch.int16, device=dev)
    L.call("pmu_conv3x3_pack_dma", w.data_ptr(), Cout, Cin, int(dgrad), wp.data_ptr(), L.stream())
    torch.cuda.synchronize()
    ref = _expected_dma(w, dgrad)
    assert ref.numel() == n
    assert torch.equal(wp.cpu(), ref.view(torch.int16))


@pytest.mark.parametrize("dgrad", [False, True])
def test_pack_dma_multi(dev, dgrad):
    """One batched launch over ragged tensors (each job's blocks from pmu_conv3x3_pack_dma_blocks) equals
    the single-tensor packs."""
    from pmu_hip import _lib as L
    shapes = [(64, 64), (40, 24), (256, 160), (96, 8), (512, 256)]
    g = torch.Generator().manual_seed(11 + int(dgrad))
    ws = [torch.randn(co, ci, 3, 3, generator=g).to(dev) for co, ci in shapes]
    outs = [torch.full((L.lib().pmu_conv3x3_packed_size_dma(co, ci, int(dgrad)) // 2,), -1, dtype=torch.int16,
                       device=dev) for co, ci in shapes]
    jobs = (L.PmuPackJob * len(ws))()
    b0 = 0
    for i, (w, o) in enumerate(zip(ws, outs)):
        nb = L.lib().pmu_conv3x3_pack_dma_blocks(w.shape[0], w.shape[1], int(dgrad))
        jobs[i] = L.PmuPackJob(w.data_ptr(), o.data_ptr(), w.shape[0], w.shape[1], b0, nb)
        b0 += nb
    jt = torch.frombuffer(bytearray(bytes(jobs)), dtype=torch.uint8).to(dev)
    L.call("pmu_conv3x3_pack_dma_multi", jt.data_ptr(), len(ws), b0, int(dgrad), L.stream())
    torch.cuda.synchronize()
    for w, o in zip(ws, outs):
        single = torch.full_like(o, -1)
        L.call("pmu_conv3x3_pack_dma", w.data_ptr(), w.shape[0], w.shape[1], int(dgrad), single.data_ptr(),
               L.stream())
        torch.cuda.synchronize()
        assert torch.equal(o, single), tuple(w.shape)
        assert torch.equal(o.cpu(), _expected_dma(w, dgrad).view(torch.int16))
