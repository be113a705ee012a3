"""In-repo KServe-v2 test / bench server (HTTP + gRPC)."""
from .app import ServerHandle, default_models, start_server  # noqa: F401
