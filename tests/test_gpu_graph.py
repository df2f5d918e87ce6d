"""GPU: HIP-graph replay of the Net forward (RRINEngine.graph / NetGraph; bench.py --graph).

The graph captures the very launches of an eager forward (rrin_net_fwd per stream part) over
static input / output / t-coefficient buffers, so its output must be the eager forward's bit for
bit: at the BASELINE C2 shape on one stream, on four streams (multi-stream capture: fork and
join inside the graph), for every t (the coefficients are rewritten in device memory before a
replay; round 1's probe baked a freed host temporary into the graph -- DESIGN.md §10), and after
the engine's workspace cache has evicted the captured shape (the graph holds its buffers)."""
import pytest
import torch

from rrin_amd import Net
from rrin_amd.synthetic import keyed_state_dict, synthetic_batch

pytestmark = pytest.mark.gpu


def make_net(dev, precision):
    net = Net()
    net.load_state_dict(keyed_state_dict(net.state_dict(), stress=True), strict=True)
    net = net.to(dev).eval()
    net.precision = precision
    return net


@pytest.mark.parametrize("precision,n,h,w,streams", [("fp32", 1, 368, 640, 1), ("fp16", 4, 64, 96, 4),
                                                     ("fp32", 3, 64, 96, 2), ("fp32_split16", 2, 96, 128, 2)])
def test_graph_replay_bitwise_eager(gpu, precision, n, h, w, streams):
    net = make_net(gpu, precision)
    eng = net.engine()
    i0, i1 = synthetic_batch(n, h, w, first_index=11)
    i0, i1 = i0.to(gpu), i1.to(gpu)
    with torch.no_grad():
        g = eng.graph(n, h, w, streams=streams)
        assert eng.graph(n, h, w, streams=streams) is g  # cached per shape and split
        g.i0.copy_(i0)
        g.i1.copy_(i1)
        for t in (0.5, 0.25, torch.linspace(0.2, 0.8, n), 0.5):
            out = g.replay(t)
            ref = eng.forward(i0, i1, t, streams=streams)
            torch.cuda.synchronize(gpu)
            assert torch.equal(out, ref), f"t={t}"
        # repeated replays with the same t are bitwise stable
        a = g.replay(0.5).clone()
        b = g.replay(0.5).clone()
        assert torch.equal(a, b)
    eng.check_range()


def test_graph_survives_workspace_eviction(gpu):
    """Enough other shapes to evict the captured shape's workspaces from the engine cache; the
    graph keeps its own references, so its replays stay correct."""
    net = make_net(gpu, "fp32")
    eng = net.engine()
    i0, i1 = synthetic_batch(2, 64, 96, first_index=5)
    i0, i1 = i0.to(gpu), i1.to(gpu)
    with torch.no_grad():
        g = eng.graph(2, 64, 96, streams=2)
        g.i0.copy_(i0)
        g.i1.copy_(i1)
        first = g.replay(0.5).clone()
        for k in range(6):   # 6 shapes x 2 parts > MAX_WORKSPACES
            a, b = synthetic_batch(2, 32 + 16 * k, 64, first_index=k)
            eng.forward(a.to(gpu), b.to(gpu), 0.5, streams=2)
        assert not any(key[1:3] == (64, 96) for key in eng._ws)
        again = g.replay(0.5)
        torch.cuda.synchronize(gpu)
        assert torch.equal(again, first)
        assert torch.equal(again, eng.forward(i0, i1, 0.5, streams=2))
