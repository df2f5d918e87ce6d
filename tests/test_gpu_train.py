"""Training path: the HIP forward / backward kernels of
csrc/train.hip through rrin_amd.autograd, against PyTorch-CPU autograd of the
reference operators (float64 per op, the CPU oracle for the whole Net).

The reference trains through Net.forward with autograd (train.py:98) and
loss.backward() (train.py:144)."""
import pytest
import torch
import torch.nn.functional as F

from rrin_amd import Net
from rrin_amd import autograd as ag
from rrin_amd.synthetic import keyed_state_dict, synthetic_batch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / max(b.abs().max(), 1e-30))


@pytest.mark.parametrize("n,cin,cout,h,w", [(2, 6, 32, 9, 13), (1, 32, 64, 16, 24), (2, 70, 4, 7, 11),
                                            (1, 64, 32, 20, 36)])
@pytest.mark.parametrize("leaky", [False, True])
def test_conv3x3_forward_backward(gpu, n, cin, cout, h, w, leaky):
    g = torch.Generator().manual_seed(cin * 100 + cout)
    x = torch.randn(n, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    b = torch.randn(cout, generator=g) * 0.1
    gy = torch.randn(n, cout, h, w, generator=g)
    xr, wr, br = (t.double().requires_grad_() for t in (x, wt, b))
    yr = F.conv2d(xr, wr, br, padding=1)
    if leaky:
        yr = F.leaky_relu(yr, 0.1)
    yr.backward(gy.double())
    xg, wg, bg = (t.to(gpu).requires_grad_() for t in (x, wt, b))
    conv = torch.nn.Conv2d(cin, cout, 3, padding=1).to(gpu)
    conv.weight, conv.bias = torch.nn.Parameter(wg), torch.nn.Parameter(bg)
    y = ag.conv3x3(xg, conv, leaky)
    y.backward(gy.to(gpu))
    assert rel(y, yr) < 1e-5
    assert rel(xg.grad, xr.grad) < 1e-5
    assert rel(conv.weight.grad, wr.grad) < 1e-5
    assert rel(conv.bias.grad, br.grad) < 1e-5


def test_conv3x3_wgrad_many_slices(gpu):
    """A weight gradient over more than one K slice (n*h*w > 4096 pixels)."""
    g = torch.Generator().manual_seed(5)
    x = torch.randn(3, 16, 40, 72, generator=g)
    wt = torch.randn(32, 16, 3, 3, generator=g) / 12
    gy = torch.randn(3, 32, 40, 72, generator=g)
    wr = wt.double().requires_grad_()
    F.conv2d(x.double(), wr, padding=1).backward(gy.double())
    conv = torch.nn.Conv2d(16, 32, 3, padding=1).to(gpu)
    conv.weight = torch.nn.Parameter(wt.to(gpu))
    ag.conv3x3(x.to(gpu), conv).backward(gy.to(gpu))
    assert rel(conv.weight.grad, wr.grad) < 1e-5


@pytest.mark.parametrize("shape", [(2, 3, 8, 12), (1, 5, 6, 10)])
def test_avg_pool2(gpu, shape):
    x = torch.randn(*shape)
    gy = torch.randn(shape[0], shape[1], shape[2] // 2, shape[3] // 2)
    xr = x.double().requires_grad_()
    F.avg_pool2d(xr, 2).backward(gy.double())
    xg = x.to(gpu).requires_grad_()
    y = ag.avg_pool2(xg)
    y.backward(gy.to(gpu))
    assert rel(y, F.avg_pool2d(x.double(), 2)) < 1e-6
    assert rel(xg.grad, xr.grad) < 1e-6


@pytest.mark.parametrize("shape", [(2, 3, 5, 7), (1, 4, 1, 3), (1, 2, 12, 20)])
def test_upsample2(gpu, shape):
    x = torch.randn(*shape)
    gy = torch.randn(shape[0], shape[1], 2 * shape[2], 2 * shape[3])
    xr = x.double().requires_grad_()
    F.interpolate(xr, scale_factor=2, mode="bilinear", align_corners=False).backward(gy.double())
    xg = x.to(gpu).requires_grad_()
    y = ag.upsample2(xg)
    y.backward(gy.to(gpu))
    assert rel(y, F.interpolate(x.double(), scale_factor=2, mode="bilinear", align_corners=False)) < 1e-6
    assert rel(xg.grad, xr.grad) < 1e-5


def _ref_warp(img, flow):  # model.py:8-21 on the CPU
    n, _, h, w = img.shape
    gy, gx = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
    x = gx.unsqueeze(0).float() + flow[:, 0]
    y = gy.unsqueeze(0).float() + flow[:, 1]
    grid = torch.stack((2 * (x / w - 0.5), 2 * (y / h - 0.5)), dim=3)
    return F.grid_sample(img, grid, mode="bilinear", padding_mode="zeros", align_corners=False)


@pytest.mark.parametrize("scale", [0.3, 4.0, 40.0])
def test_backwarp(gpu, scale):
    g = torch.Generator().manual_seed(int(scale * 10))
    img = torch.rand(2, 3, 17, 23, generator=g)
    flow = torch.randn(2, 2, 17, 23, generator=g) * scale
    go = torch.randn(2, 3, 17, 23, generator=g)
    ir, fr = img.clone().requires_grad_(), flow.clone().requires_grad_()
    out_r = _ref_warp(ir, fr)
    out_r.backward(go)
    ig, fg = img.to(gpu).requires_grad_(), flow.to(gpu).requires_grad_()
    out = ag.backwarp(ig, fg)
    out.backward(go.to(gpu))
    assert rel(out, out_r) < 1e-5
    assert rel(ig.grad, ir.grad) < 1e-5
    assert rel(fg.grad, fr.grad) < 1e-4
    # the image gradient is a scatter summed in fixed point: bitwise run to run
    ig2 = img.to(gpu).requires_grad_()
    ag.backwarp(ig2, fg.detach()).backward(go.to(gpu))
    assert torch.equal(ig.grad, ig2.grad)


@pytest.mark.parametrize("stress", [False, True])
def test_net_gradients_match_oracle_autograd(gpu, stress):
    """d(sum of Net output) / d(inputs, every parameter) through the HIP training
    path vs PyTorch-CPU autograd of the oracle (the reference op sequence),
    within 1e-4 relative (max-abs error / max-abs gradient, per tensor).

    With the stress weights (10-18 px flows) the gradient is ill-conditioned: the
    bilinear sampler's derivative jumps where a sample position crosses an
    integer, so the reference's OWN fp32 gradients move by up to ~4e-3 relative
    when its weights are perturbed by 1e-6 relative.  Each tensor's bound is
    therefore max(1e-4, 2 x that sensitivity of the oracle), measured here."""
    from oracle.ref_net import net_forward
    net = Net()
    sd = keyed_state_dict(net.state_dict(), stress=stress)
    net.load_state_dict(sd)
    net = net.to(gpu).train()
    i0, i1 = synthetic_batch(2, 64, 96, first_index=3)
    a0, a1 = i0.to(gpu).requires_grad_(), i1.to(gpu).requires_grad_()
    out = net(a0, a1, 0.5)
    out.sum().backward()

    def oracle(weights):
        p = {k: v.clone().requires_grad_() for k, v in weights.items()}
        r0, r1 = i0.clone().requires_grad_(), i1.clone().requires_grad_()
        o = net_forward(p, r0, r1, 0.5)
        o.sum().backward()
        return o, {k: v.grad for k, v in p.items()}, r0.grad, r1.grad

    ref, gref, g0, g1 = oracle(sd)
    g = torch.Generator().manual_seed(1)
    _, gpert, p0, p1 = oracle({k: v * (1 + 1e-6 * torch.randn(v.shape, generator=g)) for k, v in sd.items()})
    assert rel(out, ref) < 1e-4
    bad = []
    for name, p in net.named_parameters():
        tol = max(1e-4, 2 * rel(gpert[name], gref[name]))
        e = rel(p.grad, gref[name])
        if e > tol:
            bad.append((name, e, tol))
    assert not bad, bad
    assert rel(a0.grad, g0) <= max(1e-4, 2 * rel(p0, g0))
    assert rel(a1.grad, g1) <= max(1e-4, 2 * rel(p1, g1))


def test_net_backward_is_deterministic(gpu):
    net = Net()
    net.load_state_dict(keyed_state_dict(net.state_dict(), stress=True))
    net = net.to(gpu)
    i0, i1 = synthetic_batch(1, 32, 48)
    grads = []
    for _ in range(2):
        net.zero_grad()
        a0 = i0.to(gpu).requires_grad_()
        net(a0, i1.to(gpu), 0.3).square().mean().backward()
        grads.append([a0.grad.clone()] + [p.grad.clone() for p in net.parameters()])
    assert all(torch.equal(a, b) for a, b in zip(*grads))


@pytest.mark.parametrize("cout,cin", [(64, 32), (40, 24), (3, 13), (128, 64)])
@pytest.mark.parametrize("bm", [32, 64])
@pytest.mark.parametrize("mode", [0, 1])
def test_tpack_wino_matches_host_packing(gpu, cout, cin, bm, mode):
    """rrin_tpack_wino (device) is bitwise the host packing rrin_pack_conv3x3_wino_bm: mode 0 of
    W, mode 1 (the dgrad conv) of W transposed (ci <-> co) and flipped (ky, kx -> 2 - ky, 2 - kx);
    channel counts that are not multiples of 8 pad with zeros the same way."""
    import ctypes as C

    import numpy as np

    from rrin_amd import _lib
    lib = _lib.lib()
    torch.manual_seed(cout * 7 + cin + bm + mode)
    w = torch.randn(cout, cin, 3, 3)
    ref_w = w if mode == 0 else w.transpose(0, 1).flip(2, 3)
    rows, cols = ref_w.shape[:2]
    wn = ref_w.contiguous().numpy()
    nf = lib.rrin_pack_conv3x3_wino_bm_floats(rows, cols, bm)
    host = np.zeros(nf, np.float32)
    bp = np.zeros(lib.rrin_pack_bias_floats(rows, bm), np.float32)
    b = np.zeros(rows, np.float32)
    _lib.check(lib.rrin_pack_conv3x3_wino_bm(wn.ctypes.data, b.ctypes.data, rows, cols, bm, None, host.ctypes.data,
                                             bp.ctypes.data))
    wd = w.to(gpu).contiguous()
    dev = torch.full((nf,), float("nan"), device=gpu)
    _lib.check(lib.rrin_tpack_wino(C.c_void_p(wd.data_ptr()), cout, cin, bm, mode, C.c_void_p(dev.data_ptr()),
                                   C.c_void_p(torch.cuda.current_stream(gpu).cuda_stream)))
    torch.cuda.synchronize(gpu)
    assert torch.equal(dev.cpu(), torch.from_numpy(host))


def test_r32_buffers_per_stream_and_bounded(gpu):
    """The training convs' record buffers are cached per (stream, shape, role) and the cache is
    bounded: two streams get distinct buffers, and many shapes do not grow it."""
    a = ag._r32_buf(1, 8, 16, 32, gpu, "tx")
    s = torch.cuda.Stream(gpu)
    with torch.cuda.stream(s):
        b = ag._r32_buf(1, 8, 16, 32, gpu, "tx")
    assert a is not b and ag._r32_buf(1, 8, 16, 32, gpu, "tx") is a
    for h in range(16, 16 + 16 * (ag.R32_BUFS_MAX + 8), 16):
        ag._r32_buf(1, 8, h, 32, gpu, "ty")
    assert len(ag._R32_BUFS) <= ag.R32_BUFS_MAX
