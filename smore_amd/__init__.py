"""smore_amd -- MI355X-native (gfx950) SMORe hot path: proNet alias sampling +
fused Opt_SigmoidSGD / Opt_SGD / Opt_BPRSGD updates behind a C ABI.

The HIP shared library is required; there is no CPU fallback."""
from . import _lib  # noqa: F401  (raises ImportError if libsmore_hip.so is missing)
from .models import APP, BPR, HPE, LINE, MF, DeepWalk, Walklets  # noqa: F401
from .pronet import Group, ProNet, comm_unique_id, deepwalk_order  # noqa: F401

__all__ = ["ProNet", "Group", "LINE", "MF", "BPR", "DeepWalk", "Walklets", "APP", "HPE", "deepwalk_order", "comm_unique_id"]
