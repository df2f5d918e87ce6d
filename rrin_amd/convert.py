"""Frame interpolation of an image folder / video — the reference's convert entry
point (`/root/reference/convert.py:22-169`) on the HIP Net.

Kept from the reference (so outputs and resume behave the same):
* t schedule ``t = i / (sf + 1)`` for i = 1..sf (`convert.py:127-130`);
* output naming ``{n:09d}{ext}``: first frame copied as 1, then per pair the sf
  interpolated frames and the copied second frame (`convert.py:118-144`);
* resume: ``resume_index = (len(dest) - 1) // (sf + 1)`` when more than 5
  outputs exist (`convert.py:50-56`), restart at pair ``resume_index - 1`` with
  ``img_count = resume_index + resume_index*sf - sf`` (`convert.py:95,118`);
* frames: RGB, /255 (`ToTensor`), edge-padded on top to a multiple of 16
  (`dataloader.py:91-108`); outputs cropped back and quantised with
  ``mul(255).byte()`` truncation as ``to_pil_image`` does (`utils.py:51-58`).

Different (documented in DESIGN.md):
* frames are read in sorted order (the reference uses raw ``os.listdir`` order);
* a width that is not a multiple of 16 is edge-padded on the right (the
  reference pads the bottom by the width deficit and then fails in the U-Net);
* paths use ``os.path.join`` (the reference hard-codes Windows ``\\\\``);
* the pipeline is batched: ``batch`` pairs per call, the t-independent Flow
  U-Net once per pair for all sf values of t (``Net.interpolate``), frames
  decoded by a reader thread, outputs copied to pinned host memory
  asynchronously and written by a thread pool (the reference decodes on the
  main thread, recomputes Flow per t, syncs per frame and polls its writer
  queue every 0.1 s: `convert.py:97,130,133`, `utils.py:61-62`).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from queue import Queue

import numpy as np
import torch

IMG_EXT = (".png", ".jpg", ".jpeg", ".bmp", ".tif", ".tiff", ".webp")


def list_frames(folder):
    return sorted(f for f in os.listdir(folder) if f.lower().endswith(IMG_EXT))


def pad_amounts(width, height):
    """(top_pad, right_pad) to the next multiple of 16 (dataloader.py:91-101)."""
    right = (-width) % 16
    top = (-height) % 16
    return top, right


def load_frame(path):
    """PIL RGB -> float32 [3,H',W'] in [0,1], edge-padded (top / right) to /16."""
    from PIL import Image
    with Image.open(path) as im:
        arr = np.asarray(im.convert("RGB"), dtype=np.uint8)
    h, w = arr.shape[:2]
    top, right = pad_amounts(w, h)
    if top or right:
        arr = np.pad(arr, ((top, 0), (0, right), (0, 0)), mode="edge")
    t = torch.from_numpy(arr.copy()).permute(2, 0, 1).float().div_(255.0)
    return t, {"width": w, "height": h, "top": top, "filetype": os.path.splitext(path)[1], "path": path}


def to_uint8_image(t: torch.Tensor, meta) -> np.ndarray:
    """[3,H',W'] float -> cropped HxWx3 uint8 with to_pil_image's mul(255).byte() truncation."""
    a = t.mul(255).to(torch.uint8)  # truncation toward zero, as torchvision's to_pil_image
    a = a[:, meta["top"]:meta["top"] + meta["height"], :meta["width"]]
    return a.permute(1, 2, 0).contiguous().numpy()


def save_image(arr, path):
    from PIL import Image
    Image.fromarray(arr).save(path)


def resume_state(dest, sf):
    """(resume_index, img_count) of convert.py:50-56,118."""
    resume_index = 1
    if os.path.exists(dest) and len(os.listdir(dest)) > 5:
        resume_index = (len(os.listdir(dest)) - 1) // (sf + 1)
    return resume_index, resume_index + resume_index * sf - sf


def pair_shards(first_pair: int, n_frames: int, world: int):
    """Contiguous, balanced ranges [lo, hi) of the pair indices first_pair ..
    n_frames-2 for each rank (pair k = frames k and k+1).  Rank r reads frames
    lo .. hi: its last frame is the first frame of rank r+1's range (the one
    frame of halo a sharded consecutive-pair dataset needs, dataloader.py:152-166)."""
    n = max(n_frames - 1 - first_pair, 0)
    return [(first_pair + n * r // world, first_pair + n * (r + 1) // world) for r in range(world)]


class _Reader:
    """Decodes frames lo..hi ahead of the GPU on a thread (bounded queue); an
    exception in the thread (unreadable / corrupt image) is re-raised in the
    consumer instead of leaving it blocked."""

    def __init__(self, src, frames, lo, hi, depth):
        self.q: Queue = Queue(maxsize=depth)
        self.t = threading.Thread(target=self._run, args=(src, frames, lo, hi), daemon=True)
        self.t.start()

    def _run(self, src, frames, lo, hi):
        try:
            for k in range(lo, hi + 1):
                self.q.put(("frame", k, *load_frame(os.path.join(src, frames[k]))))
            self.q.put(("end",))
        except BaseException as e:  # noqa: BLE001 - handed to the consumer
            self.q.put(("error", e))

    def get(self):
        item = self.q.get()
        if item[0] == "error":
            raise RuntimeError(f"reading input frames failed: {item[1]!r}") from item[1]
        return None if item[0] == "end" else item[1:]


def interpolate_folder(model, src, dest, sf, batch=4, resume=False, device=None, writers=4, log=print,
                       rank=0, world=1, group=None, gather=True):
    """Interpolate every consecutive pair of frames in ``src`` into ``dest``.

    ``model`` is an ``rrin_amd.Net`` (anything with ``interpolate(i0, i1, ts)``
    returning a list of ``[N,3,H,W]`` tensors works).  Returns the frames this
    rank wrote.

    Multi-GPU (``world`` > 1, one process per GPU, ``torch.distributed``
    initialised; replaces the single-device dispatch of convert.py:90-92,110,130):
    the pairs are split into contiguous per-rank ranges (``pair_shards``); every
    step each rank interpolates up to ``batch`` of its pairs and, with
    ``gather=True``, one all-gather (RCCL over xGMI on GPUs, gloo on CPU)
    reassembles that step's frames of all ranks in rank order on every rank, and
    rank 0 writes the whole sequence.  ``gather=False`` lets every rank write its
    own frames (the file names are global, so the outputs are the same)."""
    frames = list_frames(src)
    if len(frames) < 2:
        raise ValueError(f"need at least two frames in {src}")
    if rank == 0:
        os.makedirs(dest, exist_ok=True)
    # resume state is read by every rank before anyone writes
    resume_index, img_count0 = resume_state(dest, sf) if resume else (1, 1)
    if world > 1:
        import torch.distributed as dist
        dist.barrier(group)
    os.makedirs(dest, exist_ok=True)
    first_pair = resume_index - 1
    ts = [i / (sf + 1) for i in range(1, sf + 1)]
    shards = pair_shards(first_pair, len(frames), world)
    lo, hi = shards[rank]
    writes_here = gather is False or world == 1 or rank == 0
    pool = ThreadPoolExecutor(max_workers=writers) if writes_here else None
    futures = []
    written = [0]

    def put(fn, *a):
        futures.append(pool.submit(fn, *a))
        written[0] += 1

    def base_of(k):  # file number before pair k's outputs (convert.py:118,144)
        return img_count0 + (k - first_pair) * (sf + 1)

    if img_count0 == 1 and rank == 0:
        put(shutil.copy, os.path.join(src, frames[first_pair]),
            os.path.join(dest, f"{img_count0:09d}{os.path.splitext(frames[first_pair])[1]}"))
    t0 = time.time()
    steps = max((b - a + batch - 1) // batch for a, b in shards)
    reader = _Reader(src, frames, lo, hi, 2 * batch + 2) if hi > lo else None
    prev = reader.get() if reader else None
    pending = []
    for s_ in range(steps):
        group_items = [prev] if prev is not None else []
        k0 = lo + s_ * batch
        nloc = max(0, min(batch, hi - k0))
        while len(group_items) < nloc + 1 and nloc:
            item = reader.get()
            if item is None:
                break
            group_items.append(item)
        outs = None
        if nloc:
            prev = group_items[-1]
            i0 = torch.stack([g[1] for g in group_items[:-1]])
            i1 = torch.stack([g[1] for g in group_items[1:]])
            if device is not None:
                i0 = i0.pin_memory().to(device, non_blocking=True)
                i1 = i1.pin_memory().to(device, non_blocking=True)
            with torch.no_grad():
                outs = model.interpolate(i0, i1, ts) if hasattr(model, "interpolate") else \
                    [model(i0, i1, t) for t in ts]
        metas0 = [g[2] for g in group_items[:-1]] if nloc else []
        metas1 = [g[2] for g in group_items[1:]] if nloc else []
        if world > 1 and gather:
            outs, metas0, metas1, ks = _gather_step(outs, metas0, metas1, nloc, shards, s_, batch, sf, group,
                                                    device, getattr(model, "check_range", None))
            if rank != 0:
                continue
        else:
            ks = list(range(k0, k0 + nloc))
        if not ks:
            continue
        host = []
        for o in outs:
            h = torch.empty(o.shape, dtype=o.dtype, pin_memory=device is not None)
            h.copy_(o, non_blocking=device is not None)
            host.append(h)
        ev = None
        if device is not None:
            ev = torch.cuda.Event()
            ev.record()
        pending.append((ev, host, metas0, metas1, [base_of(k) for k in ks]))
        while len(pending) > 1:  # retire the previous batch while this one computes
            _retire(pending.pop(0), sf, dest, put, model)
    while pending:
        _retire(pending.pop(0), sf, dest, put, model)
    for f in futures:
        f.result()
    if pool is not None:
        pool.shutdown(wait=True)
    log(f"rank {rank}/{world}: interpolated pairs {lo}..{hi - 1} x {sf} frames in {time.time() - t0:.2f} s")
    return written[0]


def _gather_step(outs, metas0, metas1, nloc, shards, s_, batch, sf, group, device, model_check=None):
    """All-gather of one step's interpolated frames of every rank (rank order).
    Every rank contributes a [batch, sf, 3, H, W] slot (zero-padded past its
    nloc pairs); frame metadata travels as a Python object gather.  Returns the
    frames per t, the metadata and the global pair index of every gathered pair."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    # the fp16 range guard of every rank (fp32_split16 / fp16: an overflowed
    # forward wrote NaN frames) travels with the metadata, so rank 0 never
    # writes another rank's poisoned frames and every rank raises together
    bad = None
    if outs is not None and model_check is not None:
        try:
            model_check()
        except RuntimeError as e:
            bad = str(e)
    meta_all = [None] * world
    dist.all_gather_object(meta_all, (nloc, metas0, metas1, None if outs is None else tuple(outs[0].shape[1:]),
                                      None if outs is None else outs[0].dtype, bad), group=group)
    errs = [(r, m[5]) for r, m in enumerate(meta_all) if m[5]]
    if errs:
        raise RuntimeError(f"rank {errs[0][0]}: {errs[0][1]}")
    shape = next(m[3] for m in meta_all if m[3] is not None)
    dtype = next(m[4] for m in meta_all if m[4] is not None)
    dev = device if device is not None else torch.device("cpu")
    slot = torch.zeros((batch, sf) + shape, dtype=dtype, device=dev)
    if outs is not None:
        slot[:nloc] = torch.stack(outs, 1)
    from .shard import gather_frames
    full = gather_frames(slot, group=group)                 # [world*batch, sf, 3, H, W]
    sel = [r * batch + j for r in range(world) for j in range(meta_all[r][0])]
    full = full[sel]
    outs_all = [full[:, i] for i in range(sf)]
    m0 = [m for r in range(world) for m in meta_all[r][1]]
    m1 = [m for r in range(world) for m in meta_all[r][2]]
    ks = [a + s_ * batch + j for (a, _), m in zip(shards, meta_all) for j in range(m[0])]
    return outs_all, m0, m1, ks


def _retire(item, sf, dest, put, model=None):
    ev, host, metas0, metas1, bases = item
    if ev is not None:
        ev.synchronize()
    if model is not None and hasattr(model, "check_range"):
        model.check_range(wait=False)  # fp16-stored precisions: raise instead of writing NaN frames
    for p, (m0, m1, base) in enumerate(zip(metas0, metas1, bases)):
        for i in range(sf):
            put(lambda t, m, path: save_image(to_uint8_image(t, m), path), host[i][p], m0,
                os.path.join(dest, f"{base + i + 1:09d}{m0['filetype']}"))
        put(shutil.copy, m1["path"], os.path.join(dest, f"{base + sf + 1:09d}{m1['filetype']}"))


def find_checkpoint(model_name, models_dir="models"):
    """Last checkpoint whose name starts with model_name (convert.py:100-108);
    sorted order, so Model0150.pth wins over Model0001.pth."""
    if not os.path.isdir(models_dir):
        raise TypeError(f"No model found with the name: {model_name}")
    names = [n for n in sorted(os.listdir(models_dir)) if n.lower().startswith(model_name.lower())]
    if not names:
        raise TypeError(f"No model found with the name: {model_name}")
    return os.path.join(models_dir, names[-1])


def load_net(model_name, device, precision="fp32", models_dir="models"):
    """Net with the checkpoint's {'model','optim','epoch'} state (train.py:158-161),
    loaded with torch.load(weights_only=True) — nothing in the file is executed."""
    from .model import Net
    net = Net()
    path = find_checkpoint(model_name, models_dir)
    state = torch.load(path, map_location="cpu", weights_only=True)
    net.load_state_dict(state["model"] if "model" in state else state, strict=True)
    print(f"Using model {path}.")
    net.precision = precision
    return net.to(device).eval()


def _ffmpeg(cmd):
    if shutil.which("ffmpeg") is None:
        raise RuntimeError("ffmpeg is not installed: use --image_folder (video I/O needs ffmpeg, "
                           "as in the reference convert.py:78,153-160)")
    return subprocess.call(cmd)


def convert(args):
    """CLI entry (same flags as the reference __main__.py:47-63).  Under
    ``torchrun --nproc-per-node N`` (WORLD_SIZE > 1) every process drives its
    own GPU (LOCAL_RANK), the pairs are sharded and their frames all-gathered
    over RCCL (``interpolate_folder``); rank 0 does the ffmpeg steps and the
    folder checks and broadcasts their outcome, so a failure there ends every
    rank (same message / exit code as the reference, convert.py:67-82)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1 and int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 8:
        # RCCL's streams plus the forward's two: give HIP enough hardware queues
        # that the two forward streams do not share one; read at
        # HIP init, which has not happened yet in this process
        os.environ["GPU_MAX_HW_QUEUES"] = "8"
    if args.no_cuda or not torch.cuda.is_available():
        raise RuntimeError("rrin_amd runs on ROCm GPUs only (the reference also moves the model to .cuda() "
                           "unconditionally, convert.py:110)")
    if world > 1:
        import torch.distributed as dist
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    if args.input_video is not None:
        temp = "temp_" + os.path.basename(args.input_video)
        if args.resume and not os.path.exists(temp):
            raise Exception("Did not find temp folder to resume!")
    elif args.image_folder is not None:
        temp = "temp"
    else:
        raise Exception("Missing arguments! Video or folder needs to be specified")
    inp, dest = os.path.join(temp, "input"), os.path.join(temp, "output")
    # rank 0's folder checks and frame extraction; their outcome is broadcast so
    # that a failure ends every rank (the others would otherwise wait at the
    # next collective until its timeout)
    failure = None  # (kind, message)
    if not args.resume and rank == 0:
        try:
            if os.path.exists(dest) and os.listdir(dest):
                failure = ("raise", "Folder is already in use! Did you intend to resume the progress? "
                                    "Use the --resume flag")
            elif args.input_video is not None:
                shutil.rmtree(temp, ignore_errors=True)
                os.makedirs(inp)
                if _ffmpeg(["ffmpeg", "-i", args.input_video, "-vsync", "0", os.path.join(inp, "%9d.png")]):
                    failure = ("exit", "Failed to convert video to images.")
        except Exception as e:  # noqa: BLE001 -- re-raised on every rank below
            failure = ("raise", f"{type(e).__name__}: {e}")
    if world > 1:
        box = [failure]
        dist.broadcast_object_list(box, src=0)
        failure = box[0]
    if failure is not None:
        if world > 1:
            dist.destroy_process_group()
        if failure[0] == "exit":
            print(failure[1])
            sys.exit(1)
        raise Exception(failure[1])
    src = inp if args.input_video is not None else args.image_folder
    dev = torch.device("cuda", torch.cuda.current_device())
    net = load_net(args.model_name, dev, getattr(args, "precision", "fp32"))
    t = time.time()
    interpolate_folder(net, src, dest, args.sf, batch=getattr(args, "batch", 4), resume=args.resume, device=dev,
                       rank=rank, world=world)
    if world > 1:
        dist.barrier()
    print("end=", time.time() - t)
    if rank == 0 and args.input_video is not None and args.output_video:
        if _ffmpeg(["ffmpeg", "-r", str(args.fps), "-y", "-i", os.path.join(dest, "%9d.png"), "-c:v", "libvpx-vp9",
                    "-crf", "30", "-b:v", "20M", "-pix_fmt", "yuv420p", args.output_video]):
            print("Failed to convert interpolated images to video.")
            sys.exit(1)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if args.rm and rank == 0:
        shutil.rmtree(temp, ignore_errors=True)
    print("Finished conversion")
