"""Debug probe (GPU box): which intermediate tensor first differs between a batch of 4 and a
batch of 2 holding the same frames (visualisation capture of the product path)."""
import os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "lidar-image_object-detection_-fpn_resnet-yolov8_amd", "sfa")]
import golden_cases as gc
from sfa_hip import synthetic
from test_gpu_model import make_model, _math


class G:  # minimal stand-in for the golden fixture (model weights only)
    pass


def main():
    gpu = torch.device("cuda", 0)
    golden = G()
    golden.model = np.load(os.path.join(REPO, "tests", "golden", "model_golden.npz"))
    model = make_model(golden, gpu)
    model._engine(gpu).set_math(_math("fp16x3"))
    model.capture_visualization = True
    x = torch.from_numpy(synthetic.synthetic_bev(4, 608, 608, seed=31)).to(gpu)
    with torch.no_grad():
        model(x)
        a = model.get_visualization_data()
        model(x[2:4].contiguous())
        b = model.get_visualization_data()
    for k in ("layer1", "layer2", "layer3", "layer4"):
        d = (a["backbone_features"][k][2:4] - b["backbone_features"][k]).abs().max().item()
        print(k, d)
    for i, k in enumerate(("up_level2", "up_level3", "up_level4")):
        d = (a["kfpn_features"][i][2:4] - b["kfpn_features"][i]).abs().max().item()
        print(k, d)


if __name__ == "__main__":
    main()
