"""``python -m rrin_amd --model_name M convert --sf S --fps F --image_folder D``

Same command line as the reference (`/root/reference/__main__.py:33-72`).
``train`` is parsed for compatibility but refused: the training loop and its
losses (reference ``train.py`` / ``losses.py``: AdamW, the VGG19 perceptual loss
whose weights come from the network) are out of scope.  The
model's own forward and backward do run on the HIP training kernels
(``rrin_amd.autograd``): call ``Net`` under autograd from your loop."""
import argparse
import warnings


def build_parser():
    p = argparse.ArgumentParser(description="RRIN video frame interpolation on MI355X (HIP)")
    p.add_argument("--model_name", type=str, default="Model", required=True, help="Name of model")
    p.add_argument("--no-cuda", action="store_true", default=False, help="disables CUDA")
    p.add_argument("--rm", action="store_true", default=False, help="Removed temp folder on proper finish.")
    sub = p.add_subparsers(dest="mode")
    sub.required = True
    tr = sub.add_parser("train", help="Train the model (the loop is not shipped by rrin_amd)")
    tr.add_argument("--train_folder", type=str, required=True)
    tr.add_argument("--resume", action="store_true", default=False)
    tr.add_argument("--batch_size", type=int, default=2)
    cv = sub.add_parser("convert", help="Performs interpolation of a video.")
    cv.add_argument("--input_video", type=str, required=False)
    cv.add_argument("--output_video", type=str, required=False)
    cv.add_argument("--sf", type=int, required=True, help="How many intermediate frames to make.")
    cv.add_argument("--fps", type=str, required=True, help="FPS of output")
    cv.add_argument("--image_folder", type=str, required=False)
    cv.add_argument("--resume", action="store_true", default=False)
    # rrin_amd additions
    cv.add_argument("--batch", type=int, default=4, help="frame pairs per GPU call")
    cv.add_argument("--precision", default="fp32", choices=["fp32", "fp32_split16", "fp16"],
                    help="fp32: exact fp32 (default); fp32_split16: fp32-emulated with fp16 hi+lo x3; fp16")
    return p


def main(argv=None):
    args = build_parser().parse_args(argv)
    if args.mode == "train":
        raise SystemExit("rrin_amd does not ship the training loop (AdamW, VGG19 perceptual loss: out of "
                         "scope, SURVEY §2 rows 11-12); Net.forward / backward run on the HIP training "
                         "kernels under autograd, so drive them from your own loop or the reference train.py")
    from .convert import convert
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", category=UserWarning)
        convert(args)


if __name__ == "__main__":
    main()
