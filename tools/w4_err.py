"""Max-abs error of the Winograd F(2x2) (cfg kind 3) and F(4x4) (kind 5) convs
against float64 on unit-range inputs with the keyed Net-like weights (tools
only; the tests hold kind 5 to tests/test_gpu_h8.TOL_W4)."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from rrin_amd import _lib  # noqa: E402
from rrin_amd.pp import H8Tensor  # noqa: E402
from tests.test_gpu_h8 import conv_h8, keyed_conv  # noqa: E402

dev = torch.device("cuda:0")
lib = _lib.lib()
kinds = {lib.rrin_conv_h8_cfg_wino(c): c for c in range(lib.rrin_conv_h8_cfg_count()) if lib.rrin_conv_h8_cfg_wino(c)}
for cin, cout, h, w in [(32, 32, 64, 96), (64, 64, 48, 80), (256, 256, 24, 40), (512, 512, 12, 20)]:
    torch.manual_seed(cin)
    x = torch.rand(1, cin, h, w, device=dev) * 2 - 1
    wt, b = keyed_conv(cin, cout, "err")
    ref = F.conv2d(x.double().cpu(), wt.double(), b.double(), padding=1)
    line = f"{cin:4d}->{cout:4d} {h}x{w}: |ref| max {float(ref.abs().max()):.3f}"
    for k in (3, 5):
        dst, _ = conv_h8(H8Tensor.from_nchw(x, _lib.PREC_F32R), wt, b, kinds[k], _lib.PREC_F32R)
        e = (dst.to_nchw().cpu().double() - ref).abs()
        line += f"  kind {k}: max {float(e.max()):.2e} rms {float(e.square().mean().sqrt()):.2e}"
    print(line, flush=True)
