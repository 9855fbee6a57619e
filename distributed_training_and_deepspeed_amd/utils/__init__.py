from .device import format_size, get_device, get_device_count, gpu_arch, is_rocm, local_rank  # noqa: F401
