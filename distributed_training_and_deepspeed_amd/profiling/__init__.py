from .memory import memory_status  # noqa: F401
