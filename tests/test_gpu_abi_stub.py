"""The stand-alone C-ABI stub of INTEGRATION.md §2, run verbatim: its output must
be bitwise the output of rrin_amd.Net.forward (the same rrin_net_fwd call that
the engine makes), so the documented stub cannot drift from the ABI."""
import os
import re

import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _stub_source():
    txt = open(os.path.join(REPO, "INTEGRATION.md")).read()
    m = re.search(r"<!-- stub:begin -->\s*```python\n(.*?)```\s*<!-- stub:end -->", txt, re.S)
    assert m, "INTEGRATION.md lost its stub block"
    return m.group(1)


def test_stub_block_is_parseable():
    compile(_stub_source(), "INTEGRATION.md:stub", "exec")


@pytest.mark.gpu
@pytest.mark.parametrize("t", [0.5, 0.25])
def test_integration_stub_matches_net_forward(t):
    from rrin_amd import Net
    from rrin_amd.synthetic import keyed_state_dict, synthetic_batch
    sd = keyed_state_dict(Net().state_dict())
    i0, i1 = synthetic_batch(2, 64, 96, first_index=0)
    i0, i1 = i0.cuda(), i1.cuda()
    env = {"state_dict": sd, "i0": i0, "i1": i1, "t": t}
    exec(compile(_stub_source(), "INTEGRATION.md:stub", "exec"), env)
    torch.cuda.synchronize()
    with torch.no_grad():
        ref = env["net"](i0, i1, t)
    assert torch.equal(env["out"], ref)
