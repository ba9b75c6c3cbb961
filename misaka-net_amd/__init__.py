"""misaka-net_amd -- MI355X-native batched executor for Misaka Net TIS networks.

The hot path (many independent /compute inputs through one node network) runs
in hand-written gfx950 HIP kernels behind the C ABI of include/mk.h; this
package is the host-side mirror of the reference's interface for that path.
Import name: ``misaka_net_amd`` (a symlink to this directory).
"""
from . import _native
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
