"""Shared test helpers: rebuild recipe parameters for a golden case."""
import os

import numpy as np
import torch

from crnn_hip.recipe import recipe_state_dict, synthetic_batch  # noqa: F401
import crnn_oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NUM_CLASSES = 194


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def case_params(z, num_classes=NUM_CLASSES, with_running=True):
    hidden = int(z["hidden"])
    shapes = O.param_shapes(hidden, num_classes)
    sd = recipe_state_dict(shapes, int(z["seed"]), head_gain=float(z["head_gain"]))
    if with_running:
        for k in list(z.keys()):
            if k.startswith("bn::"):
                sd[k[4:]] = torch.from_numpy(z[k])
    return sd, hidden


def pixels_to_images(pix):
    return (torch.from_numpy(np.asarray(pix)).float() / 255.0 - 0.5) / 0.5
