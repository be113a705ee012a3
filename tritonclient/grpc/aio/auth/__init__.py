"""Authentication plugins (asyncio gRPC client)."""
from ...._auth import BasicAuth

__all__ = ["BasicAuth"]
