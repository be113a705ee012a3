"""KServe-v2 REST request codec (reference tritonclient/http/_utils.py:35-150).

The JSON header is encoded compactly (no spaces), exactly like the reference's
rapidjson ``dumps``.  Unlike the reference, the request body is returned as a
list of buffers (header, then every binary input in order) so the transport
can ``writev`` it without concatenating tensors; ``_get_inference_request``
keeps the reference's ``(bytes, json_size or None)`` contract for callers such
as ``InferenceServerClient.generate_request_body``.
"""

import json
from urllib.parse import quote_plus

from tritonclient.utils import InferenceServerException, raise_error

_RESERVED = ("sequence_id", "sequence_start", "sequence_end", "priority", "binary_data_output")


def _dumps(obj):
    return json.dumps(obj, separators=(",", ":"))


def _get_error(response):
    """Return an InferenceServerException for a non-200 response, else None."""
    if response.status_code == 200:
        return None
    body = None
    try:
        body = response.read().decode("utf-8")
        error_response = (
            json.loads(body)
            if len(body)
            else {"error": "client received an empty response from the server."}
        )
        return InferenceServerException(
            msg=error_response["error"], status=str(response.status_code)
        )
    except Exception as e:
        return InferenceServerException(
            msg=f"an exception occurred in the client while decoding the response: {e}",
            status=str(response.status_code),
            debug_details=body,
        )


def _raise_if_error(response):
    error = _get_error(response)
    if error is not None:
        raise error


def _get_query_string(query_params):
    params = []
    for key, value in query_params.items():
        if isinstance(value, list):
            for item in value:
                params.append("%s=%s" % (quote_plus(key), quote_plus(str(item))))
        else:
            params.append("%s=%s" % (quote_plus(key), quote_plus(str(value))))
    return "&".join(params)


def _build_request_json(
    inputs,
    request_id,
    outputs,
    sequence_id,
    sequence_start,
    sequence_end,
    priority,
    timeout,
    custom_parameters,
):
    infer_request = {}
    parameters = {}
    if request_id != "":
        infer_request["id"] = request_id
    if sequence_id != 0 and sequence_id != "":
        parameters["sequence_id"] = sequence_id
        parameters["sequence_start"] = sequence_start
        parameters["sequence_end"] = sequence_end
    if priority != 0:
        parameters["priority"] = priority
    if timeout is not None:
        parameters["timeout"] = timeout
    infer_request["inputs"] = [i._get_tensor() for i in inputs]
    if outputs:
        infer_request["outputs"] = [o._get_tensor() for o in outputs]
    else:
        # no outputs requested: ask for every output in binary form
        parameters["binary_data_output"] = True
    if custom_parameters:
        for key, value in custom_parameters.items():
            if key in _RESERVED:
                raise_error(f'Parameter "{key}" is a reserved parameter and cannot be specified.')
            parameters[key] = value
    if parameters:
        infer_request["parameters"] = parameters
    return _dumps(infer_request).encode()


def _get_inference_request_parts(inputs, **kw):
    """Return ``(parts, json_size or None)``; parts[0] is the JSON header."""
    header = _build_request_json(inputs, **kw)
    parts = [header]
    for i in inputs:
        raw = i._get_binary_data()
        if raw is not None:
            parts.append(raw)
    if len(parts) == 1:
        return parts, None
    return parts, len(header)


def _get_inference_request(
    inputs,
    request_id,
    outputs,
    sequence_id,
    sequence_start,
    sequence_end,
    priority,
    timeout,
    custom_parameters,
):
    parts, json_size = _get_inference_request_parts(
        inputs,
        request_id=request_id,
        outputs=outputs,
        sequence_id=sequence_id,
        sequence_start=sequence_start,
        sequence_end=sequence_end,
        priority=priority,
        timeout=timeout,
        custom_parameters=custom_parameters,
    )
    if json_size is None:
        return parts[0], None
    return b"".join(bytes(p) if not isinstance(p, bytes) else p for p in parts), json_size
