"""Drop-in for the detection step of the reference demos (utils/demo_utils.py:109-127
``do_detect``, used by demo_front.py and demo_2_sides.py).

The forward, sigmoid and decode run as HIP kernels; the back view's
``torch.flip(bevmap, [1, 2])`` (demo_utils.py:110-111) is fused into the model's input
layout conversion (``SFA_IN_NCHW3_FLIP_HW``), so the GPU reads the unflipped map.  The
flipped map is still returned for drawing, as the reference returns it.

The other names the demos import from this module are host glue, restated with the
reference's behaviour: ``parse_demo_configs`` (:36-93, same flags and derived fields; the
demos set ``configs.device`` themselves, demo_front.py:53 — with ``--no_cuda`` that is the
CPU, which the gfx950 model refuses at its first forward), ``download_and_unzip`` (:96-106, needs the ``wget`` package
and the network unless the zip is already there) and ``write_credit`` (:130-137, OpenCV).
"""

from __future__ import annotations

import argparse
import os
import time
import zipfile

import numpy as np
import torch

from sfa_hip import _lib
from sfa_hip import dropin as _dropin
from utils.evaluation_utils import decode, post_processing
from utils.torch_utils import _sigmoid


class _AttrDict(dict):
    """EasyDict's attribute access (the reference builds its configs with easydict)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k) from None

    def __setattr__(self, k, v):
        self[k] = v


def make_folder(folder_name):
    """utils/misc.py:16-19."""
    if not os.path.exists(folder_name):
        os.makedirs(folder_name)


def parse_demo_configs(argv=None):
    """demo_utils.py:36-93: the demos' argparse flags and derived configuration."""
    parser = argparse.ArgumentParser(description="Demonstration config for the implementation")
    parser.add_argument("--saved_fn", type=str, default="fpn_resnet_18", metavar="FN")
    parser.add_argument("-a", "--arch", type=str, default="fpn_resnet_18", metavar="ARCH")
    parser.add_argument("--pretrained_path", type=str,
                        default="../checkpoints/fpn_resnet_18/fpn_resnet_18_epoch_300.pth",
                        metavar="PATH")
    parser.add_argument("--foldername", type=str, default="2011_09_26_drive_0014_sync", metavar="FN")
    parser.add_argument("--K", type=int, default=50)
    parser.add_argument("--no_cuda", action="store_true")
    parser.add_argument("--gpu_idx", default=0, type=int)
    parser.add_argument("--peak_thresh", type=float, default=0.2)
    parser.add_argument("--output_format", type=str, default="image", metavar="PATH")
    parser.add_argument("--output-width", type=int, default=608)
    configs = _AttrDict(vars(parser.parse_args(argv)))
    configs.pin_memory = True
    configs.distributed = False
    configs.input_size = (608, 608)
    configs.hm_size = (152, 152)
    configs.down_ratio = 4
    configs.max_objects = 50
    configs.imagenet_pretrained = False
    configs.head_conv = 64
    configs.num_classes = 3
    configs.num_center_offset = 2
    configs.num_z = 1
    configs.num_dim = 3
    configs.num_direction = 2
    configs.heads = {"hm_cen": configs.num_classes, "cen_offset": configs.num_center_offset,
                     "direction": configs.num_direction, "z_coor": configs.num_z,
                     "dim": configs.num_dim}
    configs.root_dir = "../"
    configs.dataset_dir = os.path.join(configs.root_dir, "dataset", "kitti", "demo")
    configs.calib_path = os.path.join(configs.root_dir, "dataset", "kitti", "demo", "calib.txt")
    configs.results_dir = os.path.join(configs.root_dir, "results", configs.saved_fn)
    make_folder(configs.results_dir)
    return configs


def download_and_unzip(demo_dataset_dir, download_url):
    """demo_utils.py:96-106 (the download needs the network and the ``wget`` package)."""
    filename = download_url.split("/")[-1]
    filepath = os.path.join(demo_dataset_dir, filename)
    if os.path.isfile(filepath):
        print("The dataset have been downloaded")
        return
    import wget  # the reference imports it at module top; here only when a download is due
    print("\nDownloading data for demonstration...")
    wget.download(download_url, filepath)
    print("\nUnzipping the downloaded data...")
    with zipfile.ZipFile(filepath, "r") as zip_ref:
        zip_ref.extractall(os.path.join(demo_dataset_dir, filename[:-4]))


def write_credit(img, org_author=(500, 400), text_author="github.com/maudzung", org_fps=(50, 1000),
                 fps=None):
    """demo_utils.py:130-137 (OpenCV text overlay)."""
    import cv2
    font, scale, color, thick = cv2.FONT_HERSHEY_SIMPLEX, 1, (255, 255, 255), 2
    cv2.putText(img, text_author, org_author, font, scale, color, thick, cv2.LINE_AA)
    cv2.putText(img, "Speed: {:.1f} FPS".format(fps), org_fps, font, scale, color, thick, cv2.LINE_AA)


def time_synchronized():
    torch.cuda.synchronize() if torch.cuda.is_available() else None
    return time.time()


def do_detect(configs, model, bevmap, is_front):
    """demo_utils.py:109-127: (detections of the frame, the (flipped) bevmap, fps)."""
    dev = configs.device
    x = bevmap.unsqueeze(0).to(dev, non_blocking=True).float()
    t1 = time_synchronized()
    if is_front:
        outputs = model(x)
    else:
        outputs = model.forward_layout(x, _lib.IN_NCHW3_FLIP_HW)
    outputs["hm_cen"] = _sigmoid(outputs["hm_cen"])
    outputs["cen_offset"] = _sigmoid(outputs["cen_offset"])
    detections = decode(outputs["hm_cen"], outputs["cen_offset"], outputs["direction"],
                        outputs["z_coor"], outputs["dim"], K=configs.K)
    detections = detections.cpu().numpy().astype(np.float32)
    detections = post_processing(detections, configs.num_classes, configs.down_ratio,
                                 configs.peak_thresh)
    t2 = time_synchronized()
    if not is_front:
        bevmap = torch.flip(bevmap, [1, 2])  # the returned display copy, as the reference
    return detections[0], bevmap, 1 / max(t2 - t1, 1e-9)


# names of the reference module this drop-in does not define come from the reference
__getattr__ = _dropin.module_getattr(__name__)
