"""MI355X-native CRNN hot path (SE-ResNet31 -> BiLSTM -> CTC) over libcrnn_hip.so."""
from ._lib import build, lib, F32, BF16  # noqa: F401
from .ctc import ctc_loss, ctc_greedy_decode, ctc_greedy_decoder, decode  # noqa: F401
from .optim import FusedAdamW  # noqa: F401

__version__ = "0.1.0"
