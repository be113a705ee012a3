"""Build the KServe-v2 protobuf descriptors at import time (see _protoc.py).

Registers ``model_config.proto`` and ``grpc_service.proto`` in the default
descriptor pool exactly once, then exposes every top-level message/enum as a
module-level class, mirroring what protoc-generated ``*_pb2`` modules provide.
"""

from google.protobuf import descriptor_pool, message_factory

from . import _protoc

_POOL = descriptor_pool.Default()
_FILES = {}


def _register():
    if _FILES:
        return _FILES
    files = _protoc.load_files()
    for pf in files:
        try:
            fd = _POOL.FindFileByName(pf.name)
        except KeyError:
            fd = _POOL.AddSerializedFile(
                _protoc.to_file_descriptor_proto(pf).SerializeToString()
            )
        _FILES[pf.name] = fd
    return _FILES


def populate(module_globals, file_name):
    """Fill a module namespace with the classes of one .proto file."""
    fd = _register()[file_name]
    module_globals["DESCRIPTOR"] = fd
    for name, mdesc in fd.message_types_by_name.items():
        module_globals[name] = message_factory.GetMessageClass(mdesc)
    for name, edesc in fd.enum_types_by_name.items():
        from google.protobuf.internal import enum_type_wrapper

        wrapper = enum_type_wrapper.EnumTypeWrapper(edesc)
        module_globals[name] = wrapper
        for vname, v in edesc.values_by_name.items():
            module_globals[vname] = v.number
