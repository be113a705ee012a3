"""triton-mi355x: MI355X-native KServe-v2 / Triton inference client SDK.

Drop-in replacement for the ``tritonclient`` package of the reference
(Interactions-AI/triton-client, ``src/python/library/tritonclient``):

* ``tritonclient.http`` / ``tritonclient.http.aio`` — REST + binary-tensor
* ``tritonclient.grpc`` / ``tritonclient.grpc.aio`` — gRPC unary/stream
* ``tritonclient.utils`` — dtypes, BYTES/BF16 codecs, ``shared_memory``,
  ``hip_shared_memory`` (``cuda_shared_memory`` is an alias on ROCm).
"""

__version__ = "2.51.0+mi355x"
