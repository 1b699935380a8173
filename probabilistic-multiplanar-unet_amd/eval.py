"""Volume evaluation — drop-in for PMU/eval.py (same CLI: -f/--load, -d/--dir, -m/--model).

The reference script does not parse (eval.py:137-138); this is its evident intent, restated:
predict every slice of every test scan along the three standard views, compare each view's
volume and the 3-view average against the ground truth (Dice of classes 1 and 2), and save the
averaged label volume.  Prediction is batched on resident scans and the fusion is one kernel
(predict.predict_volume / pmu_hip.fusion).
"""
import argparse
import logging
import os

import numpy as np
import torch

from predict import predict_volume
from trainer import ProbUNetTrainer, UNetTrainer
from utils.mri_dataset import MRI_Dataset


def get_args():
    parser = argparse.ArgumentParser(description="Predict using a trained UNet",
                                     formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    parser.add_argument("-f", "--load", dest="load", type=str, default=None, help="Load model from a .pth file")
    parser.add_argument("-d", "--dir", dest="dir", type=str, default=None, help="image and label superdirs.")
    parser.add_argument("-m", "--model", dest="net", type=str, default="unet", help="what model to use: unet or probunet")
    parser.add_argument("-o", "--out", dest="out", type=str, default="predictions", help="output directory")
    parser.add_argument("-b", "--batch-size", dest="batch", type=int, default=32, help="slices per launch")
    return parser.parse_args()


def save_label(label, title):
    arr = label.cpu().numpy().astype(np.float32)
    try:
        import nibabel as nib
        nib.save(nib.Nifti1Image(arr, affine=np.eye(4)), title)
    except ImportError:
        np.save(title + ".npy", arr)


def main():
    logging.basicConfig(level=logging.INFO, format="%(levelname)s: %(message)s")
    args = get_args()
    device = torch.device("cuda")
    if args.net == "unet":
        train = UNetTrainer(device, n_channels=1, n_classes=3, load_model=args.load)
    elif args.net == "probunet":
        train = ProbUNetTrainer(device, n_channels=1, n_classes=3, load_model=args.load, latent_dim=6, beta=10)
    else:
        raise SystemExit(f"Error! {args.net} is not a valid model")
    dir_img = os.path.join(args.dir, "images") if args.dir else "data/test/images"
    dir_mask = os.path.join(args.dir, "labels") if args.dir else "data/test/labels"
    dataset = MRI_Dataset(dir_img, dir_mask, train.net.n_classes, filter=False)
    os.makedirs(args.out, exist_ok=True)
    per_volume = {k: [] for k in ("view0", "view1", "view2", "average")}
    for scan in range(len(dataset.ids)):
        res = predict_volume(train.net, dataset, scan, batch_size=args.batch, prob=(args.net == "probunet"))
        d = res["dice"].cpu().numpy()
        for i, k in enumerate(per_volume):
            per_volume[k].append(d[i, 1:3])
        save_label(res["label"], os.path.join(args.out, dataset.ids[scan]))
    for k, v in per_volume.items():
        v = np.array(v)
        logging.info(f"{k}: dice mean {v.mean(0)} std {v.std(0)}")


if __name__ == "__main__":
    main()
