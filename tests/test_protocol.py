"""Wire-format checks: protoc-lite descriptors and golden HTTP request bodies.

Field numbers are pinned against hand-encoded protobuf bytes (tag = number<<3
| wiretype) so a descriptor drift breaks byte compatibility loudly."""

import json

import numpy as np

from tritonclient.grpc import model_config_pb2, service_pb2, service_pb2_grpc
from tritonclient.grpc._protoc import load_files, to_file_descriptor_proto


def _varint(n):
    out = b""
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out += bytes([b | 0x80])
        else:
            return out + bytes([b])


def _ld(field, payload):
    return _varint(field << 3 | 2) + _varint(len(payload)) + payload


def test_model_infer_request_golden_bytes():
    r = service_pb2.ModelInferRequest(model_name="m", model_version="2", id="x")
    t = r.inputs.add(name="IN", datatype="INT32", shape=[1, 4])
    r.raw_input_contents.append(b"\x01\x02")
    expect = _ld(1, b"m") + _ld(2, b"2") + _ld(3, b"x")
    tensor = _ld(1, b"IN") + _ld(2, b"INT32") + _ld(3, _varint(1) + _varint(4))
    expect += _ld(5, tensor) + _ld(7, b"\x01\x02")
    assert r.SerializeToString() == expect
    assert t.name == "IN"


def test_parameters_map_and_oneof_numbers():
    r = service_pb2.ModelInferRequest()
    r.parameters["sequence_id"].int64_param = 7
    # map entry: key=1, value=2 ; InferParameter.int64_param = 2 (varint)
    entry = _ld(1, b"sequence_id") + _ld(2, _varint(2 << 3 | 0) + _varint(7))
    assert r.SerializeToString() == _ld(4, entry)
    p = service_pb2.InferParameter(uint64_param=5)
    assert p.SerializeToString() == _varint(5 << 3) + _varint(5)
    p = service_pb2.InferParameter(double_param=1.0)
    assert p.WhichOneof("parameter_choice") == "double_param"


def test_response_and_stream_numbers():
    r = service_pb2.ModelInferResponse(model_name="a")
    r.raw_output_contents.append(b"z")
    assert r.SerializeToString() == _ld(1, b"a") + _ld(6, b"z")
    s = service_pb2.ModelStreamInferResponse(error_message="e")
    assert s.SerializeToString() == _ld(1, b"e")
    s = service_pb2.ModelStreamInferResponse(infer_response=service_pb2.ModelInferResponse(id="q"))
    assert s.SerializeToString() == _ld(2, _ld(3, b"q"))


def test_shm_register_numbers():
    r = service_pb2.CudaSharedMemoryRegisterRequest(name="n", raw_handle=b"\x00" * 64, device_id=3, byte_size=9)
    assert r.SerializeToString() == _ld(1, b"n") + _ld(2, b"\x00" * 64) + _varint(3 << 3) + _varint(3) + _varint(4 << 3) + _varint(9)
    r = service_pb2.SystemSharedMemoryRegisterRequest(name="n", key="/k", offset=1, byte_size=2)
    assert r.SerializeToString() == _ld(1, b"n") + _ld(2, b"/k") + _varint(3 << 3) + _varint(1) + _varint(4 << 3) + _varint(2)


def test_service_methods_complete():
    names = [m[0] for m in service_pb2_grpc.METHODS]
    for n in ["ServerLive", "ServerReady", "ModelReady", "ServerMetadata", "ModelMetadata", "ModelInfer",
              "ModelStreamInfer", "ModelConfig", "ModelStatistics", "RepositoryIndex", "RepositoryModelLoad",
              "RepositoryModelUnload", "SystemSharedMemoryStatus", "SystemSharedMemoryRegister",
              "SystemSharedMemoryUnregister", "CudaSharedMemoryStatus", "CudaSharedMemoryRegister",
              "CudaSharedMemoryUnregister", "TraceSetting", "LogSettings"]:
        assert n in names
    stream = [m for m in service_pb2_grpc.METHODS if m[0] == "ModelStreamInfer"][0]
    assert stream[3] and stream[4]


def test_model_config_enum_and_oneof():
    c = model_config_pb2.ModelConfig(name="d", max_batch_size=8)
    c.input.add(name="i", data_type=model_config_pb2.TYPE_FP32, dims=[3, 224, 224],
                format=model_config_pb2.ModelInput.FORMAT_NCHW)
    c.dynamic_batching.max_queue_delay_microseconds = 100
    assert c.WhichOneof("scheduling_choice") == "dynamic_batching"
    c.sequence_batching.max_sequence_idle_microseconds = 1
    assert c.WhichOneof("scheduling_choice") == "sequence_batching"
    assert model_config_pb2.TYPE_STRING == 13 and model_config_pb2.TYPE_BF16 == 14


def test_protoc_lite_roundtrip_descriptor():
    files = load_files()
    fdp = to_file_descriptor_proto(files[1])
    msgs = {m.name for m in fdp.message_type}
    assert "ModelInferRequest" in msgs and fdp.service[0].name == "GRPCInferenceService"


def test_http_request_body_golden():
    import tritonclient.http as httpclient

    a = np.arange(4, dtype=np.int32)
    i0 = httpclient.InferInput("INPUT0", [4], "INT32").set_data_from_numpy(a)
    i1 = httpclient.InferInput("INPUT1", [4], "INT32").set_data_from_numpy(a, binary_data=False)
    o = httpclient.InferRequestedOutput("OUTPUT0", binary_data=True, class_count=2)
    body, n = httpclient.InferenceServerClient.generate_request_body(
        [i0, i1], outputs=[o], request_id="7", sequence_id=3, sequence_start=True, priority=2, timeout=10,
        parameters={"custom": "v"})
    header = json.loads(body[:n])
    assert header == {
        "id": "7",
        "inputs": [
            {"name": "INPUT0", "shape": [4], "datatype": "INT32", "parameters": {"binary_data_size": 16}},
            {"name": "INPUT1", "shape": [4], "datatype": "INT32", "data": [0, 1, 2, 3]},
        ],
        "outputs": [{"name": "OUTPUT0", "parameters": {"classification": 2, "binary_data": True}}],
        "parameters": {"sequence_id": 3, "sequence_start": True, "sequence_end": False, "priority": 2,
                       "timeout": 10, "custom": "v"},
    }
    assert body[n:] == a.tobytes()
    assert b" " not in body[:n]  # compact JSON like the reference's rapidjson
    # no binary input => whole body is JSON, json_size None
    body2, n2 = httpclient.InferenceServerClient.generate_request_body([i1])
    assert n2 is None and json.loads(body2)["parameters"] == {"binary_data_output": True}


def test_http_reserved_parameter_rejected():
    import pytest

    import tritonclient.http as httpclient
    from tritonclient.utils import InferenceServerException

    i = httpclient.InferInput("x", [1], "INT32").set_data_from_numpy(np.zeros(1, np.int32))
    with pytest.raises(InferenceServerException):
        httpclient.InferenceServerClient.generate_request_body([i], parameters={"priority": 1})


def test_http_parse_response_body():
    import tritonclient.http as httpclient

    out = np.array([1.5, 2.5], dtype=np.float32)
    header = json.dumps({"model_name": "m", "model_version": "1", "outputs": [
        {"name": "o", "datatype": "FP32", "shape": [2], "parameters": {"binary_data_size": 8}},
        {"name": "j", "datatype": "INT32", "shape": [1, 2], "data": [3, 4]}]}).encode()
    r = httpclient.InferenceServerClient.parse_response_body(header + out.tobytes(), header_length=len(header))
    np.testing.assert_array_equal(r.as_numpy("o"), out)
    np.testing.assert_array_equal(r.as_numpy("j"), [[3, 4]])
    assert r.as_numpy("missing") is None
    assert r.get_output("j")["datatype"] == "INT32"
    import gzip

    r = httpclient.InferResult.from_response_body(gzip.compress(header + out.tobytes()), header_length=len(header),
                                                  content_encoding="gzip")
    np.testing.assert_array_equal(r.as_numpy("o"), out)


def test_grpc_request_builder_typed_params():
    import pytest

    import tritonclient.grpc as grpcclient
    from tritonclient.grpc._utils import _get_inference_request
    from tritonclient.utils import InferenceServerException

    i = grpcclient.InferInput("x", [2], "FP32").set_data_from_numpy(np.ones(2, np.float32))
    req = _get_inference_request("m", [i], "", "", None, "seq-1", True, False, 3, 100,
                                 {"s": "v", "b": True, "i": 4, "f": 0.5})
    assert req.parameters["sequence_id"].string_param == "seq-1"
    assert req.parameters["priority"].uint64_param == 3
    assert req.parameters["timeout"].int64_param == 100
    assert req.parameters["b"].bool_param is True and req.parameters["i"].int64_param == 4
    assert req.parameters["f"].double_param == 0.5
    assert req.raw_input_contents[0] == np.ones(2, np.float32).tobytes()
    with pytest.raises(InferenceServerException):
        _get_inference_request("m", [i], "", "", None, 0, False, False, 0, None, {"x": [1]})
