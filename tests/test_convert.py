"""Convert pipeline (rrin_amd/convert.py): naming, resume, pad/crop, t schedule.

CPU tests drive the pipeline with the CPU oracle as the model (the HIP Net needs
a GPU; the GPU test at the bottom runs the real one)."""
import os

import numpy as np
import pytest
import torch
from PIL import Image

from rrin_amd import convert as cv
from rrin_amd.synthetic import keyed_state_dict


class OracleModel:
    def __init__(self):
        from rrin_amd import Net
        self.sd = keyed_state_dict(Net().state_dict(), stress=True)
        self.calls = 0

    def interpolate(self, i0, i1, ts):
        from oracle.ref_net import net_forward
        self.calls += 1
        return [net_forward(self.sd, i0, i1, t) for t in ts]


def make_frames(folder, n, h, w, seed=0):
    os.makedirs(folder, exist_ok=True)
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    for k in range(n):
        Image.fromarray(np.roll(base, 2 * k, axis=1)).save(os.path.join(folder, f"{k + 1:09d}.png"))


def test_pad_crop_roundtrip(tmp_path):
    p = str(tmp_path / "f.png")
    arr = np.random.default_rng(1).integers(0, 256, (37, 50, 3), dtype=np.uint8)
    Image.fromarray(arr).save(p)
    t, meta = cv.load_frame(p)
    assert t.shape == (3, 48, 64)                              # padded to /16
    assert torch.equal(t[:, :11, :50], t[:, 11:12, :50].expand(3, 11, 50))  # edge-padded on top
    back = cv.to_uint8_image(t, meta)
    np.testing.assert_array_equal(back, arr)                   # k/255 * 255 truncates back to k


def test_resume_formula(tmp_path):
    d = tmp_path / "out"
    d.mkdir()
    assert cv.resume_state(str(d), 3) == (1, 1)
    for k in range(13):
        (d / f"{k:09d}.png").write_bytes(b"")
    # convert.py:54: (13 - 1) // 4 = 3 ; convert.py:118: 3 + 3*3 - 3 = 9
    assert cv.resume_state(str(d), 3) == (3, 9)


def test_interpolate_folder_matches_oracle(tmp_path):
    src, dest = str(tmp_path / "in"), str(tmp_path / "out")
    make_frames(src, 4, 32, 48)
    model = OracleModel()
    n = cv.interpolate_folder(model, src, dest, sf=2, batch=2, device=None, log=lambda *a: None)
    names = sorted(os.listdir(dest))
    assert names == [f"{k:09d}.png" for k in range(1, 11)] and n == 10   # 4 frames, 3 pairs x (2 + 1) + 1
    assert model.calls == 2                                                # batches of 2 pairs
    # originals copied at 1, 4, 7, 10
    for k, src_idx in [(1, 1), (4, 2), (7, 3), (10, 4)]:
        assert open(os.path.join(dest, f"{k:09d}.png"), "rb").read() == \
            open(os.path.join(src, f"{src_idx:09d}.png"), "rb").read()
    # frame 3 = pair (2,3) at t=1/3... check pair (1,2), t = 2/3 -> file 3
    i0, _ = cv.load_frame(os.path.join(src, f"{1:09d}.png"))
    i1, meta = cv.load_frame(os.path.join(src, f"{2:09d}.png"))
    ref = model.interpolate(i0[None], i1[None], [2 / 3])[0][0]
    got = np.asarray(Image.open(os.path.join(dest, f"{3:09d}.png")))
    np.testing.assert_array_equal(got, cv.to_uint8_image(ref, meta))


def test_interpolate_folder_resume(tmp_path):
    src, dest = str(tmp_path / "in"), str(tmp_path / "out")
    make_frames(src, 5, 32, 48)
    full = str(tmp_path / "full")
    cv.interpolate_folder(OracleModel(), src, full, sf=1, batch=3, log=lambda *a: None)
    os.makedirs(dest)
    for name in sorted(os.listdir(full))[:6]:   # pretend the first run stopped after 6 files
        os.link(os.path.join(full, name), os.path.join(dest, name))
    cv.interpolate_folder(OracleModel(), src, dest, sf=1, batch=3, resume=True, log=lambda *a: None)
    assert sorted(os.listdir(dest)) == sorted(os.listdir(full))
    for name in os.listdir(full):
        assert open(os.path.join(dest, name), "rb").read() == open(os.path.join(full, name), "rb").read()


def test_find_checkpoint_and_safe_load(tmp_path):
    from rrin_amd import Net
    md = tmp_path / "models"
    md.mkdir()
    sd = keyed_state_dict(Net().state_dict())
    torch.save({"model": sd, "optim": {}, "epoch": 2}, md / "model0001.pth")
    torch.save({"model": sd, "optim": {}, "epoch": 3}, md / "model0002.pth")
    assert cv.find_checkpoint("Model", str(md)).endswith("model0002.pth")
    with pytest.raises(TypeError):
        cv.find_checkpoint("other", str(md))


def test_cli_parses_reference_flags():
    from rrin_amd.__main__ import build_parser
    a = build_parser().parse_args(["--model_name", "M", "convert", "--sf", "3", "--fps", "60",
                                   "--image_folder", "x"])
    assert (a.model_name, a.mode, a.sf, a.fps, a.image_folder, a.resume) == ("M", "convert", 3, "60", "x", False)


@pytest.mark.gpu
def test_convert_on_gpu_matches_oracle(tmp_path, gpu):
    """End to end on the HIP Net: every interpolated PNG equals the oracle's
    frame quantised the same way, except for rare 1-LSB truncation flips."""
    from rrin_amd import Net
    src, dest = str(tmp_path / "in"), str(tmp_path / "out")
    make_frames(src, 5, 64, 96, seed=3)
    net = Net()
    net.load_state_dict(keyed_state_dict(net.state_dict(), stress=True))
    net = net.to(gpu).eval()
    cv.interpolate_folder(net, src, dest, sf=3, batch=2, device=gpu, log=lambda *a: None)
    ref = cv.interpolate_folder(OracleModel(), src, str(tmp_path / "ref"), sf=3, batch=2, log=lambda *a: None)
    assert len(os.listdir(dest)) == ref == 17
    for name in os.listdir(dest):
        a = np.asarray(Image.open(os.path.join(dest, name))).astype(int)
        b = np.asarray(Image.open(os.path.join(str(tmp_path / "ref"), name))).astype(int)
        assert np.abs(a - b).max() <= 1 and (a != b).mean() < 0.01


class BlendModel:
    """Cheap deterministic stand-in (plumbing tests): (1-t) i0 + t i1."""

    def interpolate(self, i0, i1, ts):
        return [(1 - t) * i0 + t * i1 for t in ts]


def test_reader_error_is_raised(tmp_path):
    """A frame the reader thread cannot decode surfaces as an exception in the
    caller instead of a hang (the thread hands the error over the queue)."""
    src, dest = str(tmp_path / "in"), str(tmp_path / "out")
    make_frames(src, 4, 32, 48)
    with open(os.path.join(src, f"{3:09d}.png"), "wb") as f:
        f.write(b"not a png")
    with pytest.raises(RuntimeError, match="reading input frames failed"):
        cv.interpolate_folder(BlendModel(), src, dest, sf=1, batch=2, log=lambda *a: None)


def test_pair_shards_cover_pairs_with_one_frame_halo():
    sh = cv.pair_shards(0, 11, 4)            # 10 pairs over 4 ranks
    assert sh == [(0, 2), (2, 5), (5, 7), (7, 10)]
    assert all(b == c for (_, b), (c, _) in zip(sh[:-1], sh[1:]))   # contiguous; rank r reads frame b = next lo
    assert cv.pair_shards(3, 11, 2) == [(3, 6), (6, 10)]          # resume: pairs 3..9
    assert cv.pair_shards(0, 3, 4) == [(0, 0), (0, 1), (1, 1), (1, 2)]  # fewer pairs than ranks


def _convert_worker(rank, world, port, src, dest, gather, resume):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cv.interpolate_folder(BlendModel(), src, dest, sf=2, batch=2, rank=rank, world=world, gather=gather,
                              resume=resume, log=lambda *a: None)
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("gather", [True, False])
def test_sharded_convert_equals_single_process(tmp_path, gather):
    """World-2 gloo: sharded pairs (+ all-gather to rank 0, or per-rank writes)
    give byte-identical files to the one-process run, also when resuming."""
    import socket
    import torch.multiprocessing as mp

    def port():
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        p = s.getsockname()[1]
        s.close()
        return p

    src = str(tmp_path / "in")
    make_frames(src, 8, 32, 48, seed=5)       # 7 pairs: ranks get 3 and 4
    ref = str(tmp_path / "ref")
    cv.interpolate_folder(BlendModel(), src, ref, sf=2, batch=2, log=lambda *a: None)
    dest = str(tmp_path / "out")
    mp.spawn(_convert_worker, args=(2, port(), src, dest, gather, False), nprocs=2, join=True)
    assert sorted(os.listdir(dest)) == sorted(os.listdir(ref))
    for name in os.listdir(ref):
        assert open(os.path.join(dest, name), "rb").read() == open(os.path.join(ref, name), "rb").read(), name
    # resume after 7 files: (7-1)//3 = 2 -> restart at pair 1 (convert.py:54,95,118)
    dest2 = str(tmp_path / "out2")
    os.makedirs(dest2)
    for name in sorted(os.listdir(ref))[:7]:
        os.link(os.path.join(ref, name), os.path.join(dest2, name))
    mp.spawn(_convert_worker, args=(2, port(), src, dest2, gather, True), nprocs=2, join=True)
    assert sorted(os.listdir(dest2)) == sorted(os.listdir(ref))
    for name in os.listdir(ref):
        assert open(os.path.join(dest2, name), "rb").read() == open(os.path.join(ref, name), "rb").read(), name
