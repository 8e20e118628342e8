"""fp8 KV-scale calibration on the GPU: calibrated scales, and greedy-token
agreement of the fp8-KV engine with the bf16-KV engine (same weights) with
uncalibrated (1.0) and calibrated scales.

  python -m tools.kv_calib_check
"""
from dynamo_exp_amd.engine.engine import EngineConfig, LLMEngine
from tests.test_kv_fp8 import _gen


def main():
    kw = dict(model="small", device="cuda:0", block_size=64, max_model_len=2048, num_gpu_blocks=256, max_num_seqs=8,
              graph_sizes=(1, 2, 4, 8))
    prompts = [list(range(10 + i, 300 + 41 * i)) for i in range(4)]
    eb = LLMEngine(EngineConfig(**kw))
    eb.warmup()
    ref = _gen(eb, prompts, 8)
    for calib in (False, True):
        e8 = LLMEngine(EngineConfig(kv_cache_dtype="fp8", **kw), model=eb.model)
        sc = e8.calibrate_kv_scales(prompts) if calib else e8.model.kv_scales
        e8.warmup()
        got = _gen(e8, prompts, 8)
        same = sum(x == y for ra, rb in zip(got, ref) for x, y in zip(ra, rb))
        print(f"calibrated={calib} scales={sc} same={same}/32 first_tokens_same={sum(a[0] == b[0] for a, b in zip(got, ref))}/4", flush=True)
        e8.model.kv_scales = (1.0, 1.0)


if __name__ == "__main__":
    main()
