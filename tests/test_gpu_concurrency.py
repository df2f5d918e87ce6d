"""GPU: a Net forward is bitwise the same whether or not other kernels run beside
it on another HIP stream (multi-stream batch split, the RCCL all-gather of the
multi-GPU bench, or any user work).

Regression for DESIGN.md §9: built with packed FP32 VALU ops, the sub-pixel
ring fix-up's v_pk_fma_f32 results came out perturbed (low element, lanes
48-63) while an LDS-DMA conv looped on a side stream; the trigger is the
op_sel:[0,1,0] form (low result reading src1's high half).  The library is
built without packed FP32 ops (Makefile NOPK).  RRIN_CONC_ROUNDS raises the
number of rounds (3 forwards each) for the experiment scripts."""
import ctypes as C
import os

import pytest
import torch

from rrin_amd import Net, _lib
from rrin_amd.pp import H8Tensor
from rrin_amd.synthetic import keyed_state_dict, synthetic_batch
from tests.test_gpu_h8 import pack_h8

pytestmark = pytest.mark.gpu


def side_conv(dev, prec):
    """A 256->256 LDS-DMA conv on a 32x32 grid: few workgroups, so the Net's kernels
    share CUs with it."""
    lib = _lib.lib()
    n, h, w, cin, cout = 2, 32, 32, 256, 256
    cfg = next(c for c in range(lib.rrin_conv_h8_cfg_count()) if lib.rrin_conv_h8_cfg_fits(c, prec, cin))
    x = H8Tensor.from_nchw(torch.rand(n, cin, h, w, device=dev) * 2 - 1, prec)
    dst = H8Tensor(n, cout, h, w, dev, prec)
    wt = torch.randn(cout, cin, 3, 3) / (3 * cin ** 0.5)
    whi, wlo, bp, inv = pack_h8(wt, torch.zeros(cout), cfg, prec, dev)
    d = _lib.ConvH8Desc()
    d.n, d.cin, d.cout, d.cfg, d.prec, d.epi_mode, d.slope, d.inv_wscale = n, cin, cout, cfg, prec, 1, 0.1, inv
    d.src, d.dst = x.chunk_view(0, cin), dst.view(0, cout)
    d.whi, d.wlo, d.bias = whi.data_ptr(), wlo.data_ptr(), bp.data_ptr()
    return lib, d, (x, dst, whi, wlo, bp)


@pytest.mark.parametrize("precision", ["fp16", "fp32_split16", "fp32"])
def test_forward_bitwise_beside_side_stream_conv(gpu, precision):
    net = Net()
    net.load_state_dict(keyed_state_dict(net.state_dict(), stress=True), strict=True)
    net = net.to(gpu).eval()
    net.precision = precision
    net.subpixel_max_level = 0  # every sub-pixel up conv and ring fix-up, down to level 0
    eng = net.engine()
    i0, i1 = synthetic_batch(2, 128, 128, first_index=21)
    i0, i1 = i0.to(gpu), i1.to(gpu)
    lib, d, keep = side_conv(gpu, _lib.PRECISIONS["fp16" if precision == "fp32" else precision])
    side = torch.cuda.Stream(gpu)
    main = torch.cuda.current_stream(gpu)
    with torch.no_grad():
        ref = eng.forward(i0, i1, 0.5)
        torch.cuda.synchronize(gpu)
        bad = 0
        rounds = int(os.environ.get("RRIN_CONC_ROUNDS", "6"))  # tools/gpu_pk.sh raises it
        for _ in range(rounds):
            side.wait_stream(main)
            st = C.c_void_p(side.cuda_stream)
            for _ in range(150):
                _lib.check(lib.rrin_conv3x3_h8_fwd(C.byref(d), st))
            outs = [eng.forward(i0, i1, 0.5) for _ in range(3)]
            torch.cuda.synchronize(gpu)
            bad += sum(int(not torch.equal(o, ref)) for o in outs)
    assert bad == 0, f"{bad}/{3 * rounds} forwards differ from the serial result"
