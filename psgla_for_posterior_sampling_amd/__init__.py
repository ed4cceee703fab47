"""MI355X (gfx950) hot path of PSGLA / PnP-ULA posterior sampling.

Drop-in for the reference's restoration_algorithms.psgla (:163) and pnpula (:38); the
Langevin step runs in the HIP library libpsgla_hip.so (include/psgla_hip.h)."""
from .restoration_algorithms import pnpula, psgla

__all__ = ["psgla", "pnpula"]
