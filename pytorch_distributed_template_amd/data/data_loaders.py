"""Reference-named module (``/root/reference/data_loader/data_loaders.py``):
the loaders selectable by ``*_loader.type`` in config."""
from .mnist import MnistDataLoader  # noqa: F401
from .synthetic import SyntheticImageLoader, SyntheticImageNetLoader  # noqa: F401
