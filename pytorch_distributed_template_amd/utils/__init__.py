from .util import ensure_dir, read_json, write_json, inf_loop, prepare_device, MetricTracker  # noqa: F401
