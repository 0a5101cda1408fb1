"""pvamd — host-side mirror of the reference's PhaseVocoder interface over libpv.so
(the MI355X HIP phase-vocoder hot path).  See DESIGN.md and include/pv.h."""
from ._lib import PVError, frame_count, lib  # noqa: F401
from .vocoder import (PITCH_SHIFT, REF_COMPAT, STANDARD, TIME_SHIFT,  # noqa: F401
                      PhaseVocoder)
from .realtime import RealTimeVocoder  # noqa: F401
from .harmonizer import Harmonizer  # noqa: F401

__all__ = ["PhaseVocoder", "PVError", "TIME_SHIFT", "PITCH_SHIFT", "REF_COMPAT", "STANDARD", "RealTimeVocoder", "Harmonizer",
           "frame_count", "lib"]
