/* C ABI for external engines to publish KV-cache events to the router
 * (reference lib/bindings/c/src/lib.rs:52-297, consumed by the patched vLLM's
 * KVCacheEventManager).  Link against libdynamo_llm_capi.so.
 *
 * The library connects to the control plane named by $DX_CONTROL_PLANE
 * (host:port, default 127.0.0.1:4850) and publishes RouterEvents on
 * `namespace.{ns}.component.{component}.kv_events`, the subject the KV router
 * indexes.  Block content hashes use xxh3-64 over the little-endian u32 token
 * ids with seed 1337, identical to the router.  Calls are thread-safe. */
#ifndef DYNAMO_EXP_AMD_KV_EVENTS_H
#define DYNAMO_EXP_AMD_KV_EVENTS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  DYNAMO_OK = 0,
  DYNAMO_ERR = 1,
} dynamo_llm_result_t;

/* One publisher per process. worker_id is the instance (lease) id the router
 * knows the engine by; kv_block_size the engine's tokens per block. */
dynamo_llm_result_t dynamo_llm_init(const char* namespace_, const char* component, int64_t worker_id,
                                    uint32_t kv_block_size);

dynamo_llm_result_t dynamo_llm_shutdown(void);

/* Stored: num_blocks blocks whose tokens are laid out back to back in
 * token_ids (num_block_tokens[i] tokens for block i); block_ids are the
 * engine's sequence hashes of those blocks; parent_hash the sequence hash of
 * the block preceding the first one (NULL for a root chain).  Blocks that are
 * not full (num_block_tokens[i] != kv_block_size) and everything after them
 * are dropped, as the router only indexes full blocks. lora_id is reserved. */
dynamo_llm_result_t dynamo_kv_event_publish_stored(uint64_t event_id, const uint32_t* token_ids,
                                                   const size_t* num_block_tokens, const uint64_t* block_ids,
                                                   size_t num_blocks, const uint64_t* parent_hash,
                                                   uint64_t lora_id);

dynamo_llm_result_t dynamo_kv_event_publish_removed(uint64_t event_id, const uint64_t* block_ids,
                                                    size_t num_blocks);

#ifdef __cplusplus
}
#endif
#endif
