from .spawn import free_port, launch, under_launcher  # noqa: F401
