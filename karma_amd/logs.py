"""Logger with the reference's format and sinks (karma/logs.py:1-22).

stdout for INFO+, `karma.log` in the working directory for WARNING+; the file
is only created when the first warning is written (delay=True)."""
import logging

logger = logging.getLogger("karma.logs")
if not logger.handlers:
    logger.setLevel(logging.INFO)
    _fmt = logging.Formatter("{asctime} [{levelname}]: {message}", datefmt="%Y-%m-%d %H:%M:%S", style="{")
    _fh = logging.FileHandler("karma.log", delay=True)
    _fh.setFormatter(_fmt)
    _fh.setLevel(logging.WARNING)
    logger.addHandler(_fh)
    _sh = logging.StreamHandler()
    _sh.setFormatter(_fmt)
    logger.addHandler(_sh)
