"""MI355X-native EGGROLL ES engine (drop-in for HyperscaleES_T2I's ES hot path)."""
import os as _os

# MIOpen's Find (torch.backends.cudnn.benchmark) otherwise times the reference "naive" direct-conv
# solver on every DC-AE conv shape: ~250 s of warmup at 1024 px for a solver that never wins.
_os.environ.setdefault("MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD", "0")
