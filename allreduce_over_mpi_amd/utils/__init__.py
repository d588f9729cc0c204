from .perf import algbw_gbps, busbw_factor, busbw_gbps, human_bytes  # noqa: F401
