"""Device p50 of the reference pipeline, alternating runs (A/B of an env switch set by the caller)."""
import json
import sys

sys.path.insert(0, ".")
from bench import scalar_pipeline_p50  # noqa: E402

p50, mean = scalar_pipeline_p50(int(sys.argv[1]) if len(sys.argv) > 1 else 2000, "cuda")
print(json.dumps({"p50_us": round(p50, 2), "mean_us": round(mean, 2)}), flush=True)
