from .util import ensure_dir, read_json, write_json, inf_loop, MetricTracker  # noqa: F401
