"""Mocked unit tests of the HTTP client's request/error plumbing, no server
(parity with reference src/python/library/tests/test_inference_server_client.py,
which patches geventhttpclient's response; our transport's ``Response`` and
connection pool are patched instead)."""

import json
from unittest.mock import MagicMock, patch

import pytest

from tritonclient.http import InferenceServerClient
from tritonclient.http._transport import Response
from tritonclient.http._utils import _raise_if_error
from tritonclient.utils import InferenceServerException

JSON_ERROR = b'{"error":"foo","status_code":"404"}'


def _resp(code, body, headers=None):
    return Response(code, "X", dict(headers or {}), body)


@patch("tritonclient.http.InferenceServerClient._get", MagicMock(return_value={"status_code": 200}))
def test_get_method_success():
    c = InferenceServerClient("dummy_url")
    assert c._get("dummy_url", None, None)["status_code"] == 200


@patch("tritonclient.http.InferenceServerClient._post", MagicMock(return_value={"status_code": 200}))
def test_post_method_success():
    c = InferenceServerClient("dummy_url")
    assert c._post("dummy_url", "dummy_body", None, None)["status_code"] == 200


def test_json_error_body_raises_with_message_and_status():
    with pytest.raises(InferenceServerException) as ei:
        _raise_if_error(_resp(400, JSON_ERROR))
    assert ei.value.message() == "foo" and ei.value.status() == "400"


def test_plain_text_error_is_inference_server_exception_not_json_error():
    with pytest.raises(InferenceServerException) as ei:
        _raise_if_error(_resp(404, b"error_string"))
    assert ei.value.status() == "404"
    assert ei.value.debug_details() == "error_string"


def test_empty_error_body():
    with pytest.raises(InferenceServerException) as ei:
        _raise_if_error(_resp(500, b""))
    assert "empty response" in ei.value.message()


def test_200_is_not_an_error():
    _raise_if_error(_resp(200, b"{}"))


def test_control_plane_through_mocked_pool():
    """Control-plane calls go through the pool's request(): a mocked pool sees
    the exact method/URI/body, and JSON bodies are decoded."""
    c = InferenceServerClient("localhost:1")
    pool = MagicMock()
    c._pool = pool
    pool.request.return_value = _resp(200, json.dumps({"name": "srv", "version": "1"}).encode())
    assert c.get_server_metadata() == {"name": "srv", "version": "1"}
    method, uri = pool.request.call_args[0][:2]
    assert method == "GET" and uri == "/v2"
    pool.request.return_value = _resp(200, b"")
    assert c.is_server_ready() is True
    assert pool.request.call_args[0][1] == "/v2/health/ready"
    pool.request.return_value = _resp(200, b"")
    c.unload_model("m", unload_dependents=True)
    method, uri, parts = pool.request.call_args[0][:3]
    assert method == "POST" and uri == "/v2/repository/models/m/unload"
    assert json.loads(b"".join(bytes(p) for p in parts)) == {"parameters": {"unload_dependents": True}}
    pool.request.return_value = _resp(400, JSON_ERROR)
    with pytest.raises(InferenceServerException, match="foo"):
        c.get_model_metadata("m")
