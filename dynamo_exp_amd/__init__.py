"""dynamo_exp_amd -- an MI355X-native disaggregated LLM serving framework.

Layers (bottom-up):
  csrc/kernels   hand-written gfx950 HIP kernels (attention, norm, rope, sampling, KV copy)
  csrc/runtime   native C++ runtime pieces (xxh3 hashing, radix KV indexer, block pool, codec)
  ops, models    kernel wrappers and the first-party Llama model
  engine         paged-KV continuous-batching engine with hipGraph decode
  parallel       tensor parallel (RCCL + one-shot xGMI all-reduce), KV transfer over RCCL
  runtime        distributed runtime: control plane, namespaces/components/endpoints, leases
  llm            OpenAI protocols, preprocessor, backend, HTTP frontend, KV router, disagg router
  sdk, planner   `serve` graphs, service decorators, load-based planner
  cli            run / serve / llmctl / http / router / metrics entry points
"""
__version__ = "0.1.0"
