"""MI355X-native nonce search for the 15-440 distributed bitcoin miner.

Hot path: the reference miner's min-scan over bitcoin.Hash
(/root/reference/project2/bitcoin/miner/miner.go:58-65, bitcoin/hash.go:11-15),
re-built as gfx950 HIP kernels behind the C ABI in include/btcminer.h
(libbtcminer.so, built in-tree from csrc/).

    from distributed_bitcoin_minter_amd import Miner, bitcoin
    with Miner() as m:
        print(m.search("bradfitz", 0, 9999))   # (1419516646206828, 9898)
"""
from . import bitcoin, dist
from ._lib import BtcMinerError, Context, LIB_PATH, device_count, plan_segments, rccl_unique_id
from .miner import Miner

__all__ = ["bitcoin", "dist", "Miner", "Context", "BtcMinerError", "LIB_PATH", "device_count", "plan_segments",
           "rccl_unique_id"]
