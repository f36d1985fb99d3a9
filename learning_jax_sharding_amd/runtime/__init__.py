from .devices import (  # noqa: F401
    Device,
    devices,
    local_devices,
    device_count,
    local_device_count,
    process_index,
    process_count,
    default_backend,
    is_distributed,
    reset_backend,
    initialize_distributed,
    get_device,
)
