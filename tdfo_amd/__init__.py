"""tdfo_amd — an MI355X-native (gfx950/CDNA4) distributed recommender
training framework with the capabilities of massquantity/tdfo.

Layers:
  config      superset ``config.toml`` loader (reference TOMLs load verbatim)
  ops         hand-written HIP kernels (torch.ops.tdfo.*) + fp32 torch oracles
  sparse      table-batched embeddings, KeyedJaggedTensor, sharding planner
  parallel    process groups (RCCL / gloo), all-to-all dists, bucketed DP
  models      DLRM, DCN-v2, TwoTower, Bert4Rec
  data        synthetic Criteo generator (C++), Goodreads ETL, loaders
  train       explicit-step engines (hipGraph-captured) and trainer loops
  utils       checkpoints (Flax msgpack / .pth / sharded), metrics, logging
"""
__version__ = "0.1.0"
