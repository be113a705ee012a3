"""HTTP Basic authentication plugin (reference tritonclient/_auth.py:33-45)."""
import base64

from ._plugin import InferenceServerClientPlugin


class BasicAuth(InferenceServerClientPlugin):
    """Adds ``authorization: Basic <b64(user:pass)>`` to every request."""

    def __init__(self, username, password):
        token = base64.b64encode(
            username.encode("ascii") + b":" + password.encode("ascii")
        )
        self._auth_string = "Basic " + token.decode("ascii").strip()

    def __call__(self, request):
        request.headers["authorization"] = self._auth_string
