"""GPU allocation for graph workers (reference cli/allocator.py, NVML ->
here ROCm device enumeration + HIP_VISIBLE_DEVICES).

Each worker of a service with `resources: {gpu: n}` gets n whole GPUs;
fractional requests (< 1) share a GPU (packing).  Disable with
DYN_DISABLE_AUTO_GPU_ALLOCATION=1.
"""
from __future__ import annotations

import os
import shutil
import subprocess


def discover_gpus() -> list[int]:
    env = os.environ.get("DX_NUM_GPUS")
    if env is not None:
        return list(range(int(env)))
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
    if vis:
        return [int(x) for x in vis.split(",") if x.strip()]
    try:
        import torch  # device_count() does not initialise the GPU on this image

        return list(range(torch.cuda.device_count()))
    except Exception:
        pass
    if shutil.which("rocm-smi"):
        try:
            out = subprocess.run(["rocm-smi", "--showid"], capture_output=True, text=True, timeout=10).stdout
            return sorted({int(l.split("]")[0].split("[")[1]) for l in out.splitlines() if l.startswith("GPU[")})
        except Exception:
            pass
    return []


class ResourceAllocator:
    def __init__(self, gpus: list[int] | None = None):
        self.gpus = list(gpus if gpus is not None else discover_gpus())
        self.used: dict[int, float] = {g: 0.0 for g in self.gpus}

    def free_gpus(self) -> list[int]:
        return [g for g in self.gpus if self.used[g] == 0.0]

    def assign_gpus(self, count: float) -> list[int]:
        if count <= 0 or os.environ.get("DYN_DISABLE_AUTO_GPU_ALLOCATION"):
            return []
        if count < 1:
            for g in self.gpus:
                if self.used[g] + count <= 1.0 + 1e-9:
                    self.used[g] += count
                    return [g]
            raise RuntimeError("no GPU capacity left for a fractional request")
        n = int(count)
        free = self.free_gpus()
        if len(free) < n:
            raise RuntimeError(f"requested {n} GPUs, only {len(free)} free of {len(self.gpus)}")
        got = free[:n]
        for g in got:
            self.used[g] = 1.0
        return got

    def release(self, gpus: list[int], count: float = 1.0) -> None:
        for g in gpus:
            self.used[g] = max(0.0, self.used[g] - (count if count < 1 else 1.0))

    @staticmethod
    def env_for(gpus: list[int]) -> dict[str, str]:
        if not gpus:
            return {}
        v = ",".join(map(str, gpus))
        return {"HIP_VISIBLE_DEVICES": v}
