"""misaka-net_amd -- MI355X-native batched executor for Misaka Net TIS networks.

The hot path (many independent /compute inputs through one node network) runs
in hand-written gfx950 HIP kernels behind the C ABI of include/mk.h; this
package is the host-side mirror of the reference's interface for that path.
Import name: ``misaka_net_amd`` (a symlink to this directory).
"""
import os as _os
import sys as _sys

from . import _native

# Load the native library now, before PyTorch is imported: the HIP runtime,
# hiprtc and comgr it links (this ROCm's, /opt/rocm) become the process's, and
# PyTorch's bundled copies -- the same sonames -- resolve to them, so the
# native tier's modules are compiled in process by the hiprtc of the runtime
# that runs them.  Imported after PyTorch, the package still works: modules
# are then compiled by the mk_rtc helper process (this ROCm's hiprtc) and run
# by PyTorch's bundled runtime -- a pairing after which the host heap was
# found corrupted at exit on dynamic-stack networks.
if "torch" not in _sys.modules and _os.path.exists(_native.LIB_PATH):
    _native.lib()

from .network import (
    BatchResult,
    Network,
    NodeSpec,
    SessionSet,
    TisParseError,
    generate_inputs_device,
    tokenize,
    valu_probe_device,
)
from . import dist, master, networks

__all__ = [
    "BatchResult",
    "Network",
    "NodeSpec",
    "SessionSet",
    "TisParseError",
    "generate_inputs_device",
    "tokenize",
    "valu_probe_device",
    "networks",
    "dist",
    "master",
    "_native",
]
