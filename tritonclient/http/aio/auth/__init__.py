"""Authentication plugins (asyncio HTTP client)."""
from ...._auth import BasicAuth

__all__ = ["BasicAuth"]
