"""Shared client base: single-plugin registry (reference tritonclient/_client.py:31-85)."""
from tritonclient.utils import raise_error


class InferenceServerClientBase:
    """Base of every protocol client; owns the (at most one) plugin."""

    def __init__(self):
        self._plugin = None

    def _call_plugin(self, request):
        if self._plugin is not None:
            self._plugin(request)

    def register_plugin(self, plugin):
        """Register ``plugin``; raises if one is already registered."""
        if self._plugin is not None:
            raise_error(
                "A plugin is already registered. Please unregister the "
                "previous plugin first before registering a new plugin."
            )
        self._plugin = plugin

    def plugin(self):
        """Return the registered plugin or None."""
        return self._plugin

    def unregister_plugin(self):
        """Remove the registered plugin; raises if there is none."""
        if self._plugin is None:
            raise_error("No plugin has been registered.")
        self._plugin = None
