"""grpcio stub / servicer for ``inference.GRPCInferenceService``.

Hand-written equivalent of grpc_tools output: the method table is derived from
the parsed service descriptor so it always matches grpc_service.proto.
"""
import grpc

from . import service_pb2

_SERVICE = service_pb2.DESCRIPTOR.services_by_name["GRPCInferenceService"]
SERVICE_NAME = _SERVICE.full_name


def _cls(desc):
    return getattr(service_pb2, desc.name) if desc.file is service_pb2.DESCRIPTOR else _nested(desc)


def _nested(desc):
    from google.protobuf import message_factory

    return message_factory.GetMessageClass(desc)


METHODS = [
    (
        m.name,
        _cls(m.input_type),
        _cls(m.output_type),
        m.client_streaming,
        m.server_streaming,
    )
    for m in _SERVICE.methods
]


class GRPCInferenceServiceStub:
    """Client stub: one callable attribute per RPC (same names as protoc's)."""

    def __init__(self, channel):
        for name, req, resp, cs, ss in METHODS:
            path = "/%s/%s" % (SERVICE_NAME, name)
            if cs and ss:
                factory = channel.stream_stream
            elif cs:
                factory = channel.stream_unary
            elif ss:
                factory = channel.unary_stream
            else:
                factory = channel.unary_unary
            setattr(
                self,
                name,
                factory(
                    path,
                    request_serializer=req.SerializeToString,
                    response_deserializer=resp.FromString,
                ),
            )


class GRPCInferenceServiceServicer:
    """Base servicer: every RPC answers UNIMPLEMENTED unless overridden."""


def _unimplemented(name):
    def handler(self, request, context):
        context.set_code(grpc.StatusCode.UNIMPLEMENTED)
        context.set_details("Method %s not implemented!" % name)
        raise NotImplementedError("Method %s not implemented!" % name)

    return handler


for _name, *_rest in METHODS:
    setattr(GRPCInferenceServiceServicer, _name, _unimplemented(_name))


def add_GRPCInferenceServiceServicer_to_server(servicer, server):
    handlers = {}
    for name, req, resp, cs, ss in METHODS:
        fn = getattr(servicer, name)
        if cs and ss:
            h = grpc.stream_stream_rpc_method_handler
        elif cs:
            h = grpc.stream_unary_rpc_method_handler
        elif ss:
            h = grpc.unary_stream_rpc_method_handler
        else:
            h = grpc.unary_unary_rpc_method_handler
        handlers[name] = h(
            fn,
            request_deserializer=req.FromString,
            response_serializer=resp.SerializeToString,
        )
    server.add_generic_rpc_handlers(
        (grpc.method_handlers_generic_handler(SERVICE_NAME, handlers),)
    )
