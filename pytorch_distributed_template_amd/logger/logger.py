"""Logging setup (reference: ``/root/reference/logger/logger.py:7-22`` and
``logger/logger_config.json``).

Same handlers and formats (console ``%(message)s``; rotating ``info.log``,
10 MiB x 20, ``%(asctime)s - %(name)s - %(levelname)s - %(message)s``).
The reference's JSON ships as ``logger/logger_config.json`` in this package
(same schema; edit it to change handlers/levels) and is the default config.
Differences: the default path is resolved relative to this package instead of
the CWD (the reference's ``logger/logger_config.json`` only worked from the repo
root); ``default_log_config()`` is the built-in equivalent used if the file is
missing; non-zero ranks get console-only logging at WARNING so a multi-rank run
writes one ``info.log``.
"""
import logging
import logging.config
from pathlib import Path

from ..utils.util import read_json



def default_log_config():
    """Handler/formatter dict equivalent to the reference's logger_config.json."""
    return {
        "version": 1,
        "disable_existing_loggers": False,
        "formatters": {
            "simple": {"format": "%(message)s"},
            "datetime": {"format": "%(asctime)s - %(name)s - %(levelname)s - %(message)s"},
        },
        "handlers": {
            "console": {"class": "logging.StreamHandler", "level": "DEBUG",
                        "formatter": "simple", "stream": "ext://sys.stdout"},
            "info_file_handler": {"class": "logging.handlers.RotatingFileHandler", "level": "INFO",
                                  "formatter": "datetime", "filename": "info.log",
                                  "maxBytes": 10 * 1024 * 1024, "backupCount": 20, "encoding": "utf8"},
        },
        "root": {"level": "INFO", "handlers": ["console", "info_file_handler"]},
    }


DEFAULT_LOG_CONFIG = Path(__file__).resolve().parent / "logger_config.json"


def setup_logging(save_dir, log_config=DEFAULT_LOG_CONFIG, default_level=logging.INFO, rank: int = 0):
    if rank != 0:
        logging.basicConfig(level=logging.WARNING, format="[rank%d] %%(message)s" % rank, force=True)
        return
    if log_config is None:
        config = default_log_config()
    elif Path(log_config).is_file():
        config = read_json(log_config)
    else:
        config = None
    if config is not None:
        for _, handler in config["handlers"].items():
            if "filename" in handler:
                handler["filename"] = str(Path(save_dir) / handler["filename"])
        logging.config.dictConfig(config)
    else:
        print("Warning: logging configuration file is not found in {}.".format(log_config))
        logging.basicConfig(level=default_level)
