"""Backend model interface of the in-repo KServe-v2 server."""

import numpy as np

from tritonclient.grpc import model_config_pb2 as mc

from .types import OutputTensor, ServerError

_DT_TO_CFG = {
    "BOOL": mc.TYPE_BOOL,
    "UINT8": mc.TYPE_UINT8,
    "UINT16": mc.TYPE_UINT16,
    "UINT32": mc.TYPE_UINT32,
    "UINT64": mc.TYPE_UINT64,
    "INT8": mc.TYPE_INT8,
    "INT16": mc.TYPE_INT16,
    "INT32": mc.TYPE_INT32,
    "INT64": mc.TYPE_INT64,
    "FP16": mc.TYPE_FP16,
    "FP32": mc.TYPE_FP32,
    "FP64": mc.TYPE_FP64,
    "BYTES": mc.TYPE_STRING,
    "BF16": mc.TYPE_BF16,
}
CFG_TO_DT = {v: k for k, v in _DT_TO_CFG.items()}


def cfg_dtype(dt):
    return _DT_TO_CFG[dt]


class TensorSpec:
    def __init__(self, name, datatype, dims, fmt=None, label_filename="", optional=False):
        self.name = name
        self.datatype = datatype
        self.dims = list(dims)
        self.fmt = fmt
        self.label_filename = label_filename
        self.optional = optional


class Model:
    """Base class: subclasses set the class attributes and implement execute.

    ``execute(requests)`` receives a list of InferRequest (one batch) and must
    return a list (same length) whose items are either a list of OutputTensor
    or an Exception for that request.  Decoupled models implement
    ``execute_decoupled(request, emit)`` instead and call ``emit(outputs)``
    zero or more times.
    """

    name = "model"
    platform = "python"
    backend = "python"
    versions = (1,)
    max_batch_size = 0
    inputs = ()
    outputs = ()
    decoupled = False
    dynamic_batching = None  # dict(preferred=[...], max_queue_delay_us=N)
    sequence_batching = False
    ensemble_steps = None  # list of (model_name, input_map, output_map)
    instance_kind = "KIND_CPU"
    instance_count = 1
    gpus = ()
    labels = None  # list of class labels for classification outputs

    def __init__(self, version=1, **kwargs):
        self.version = version
        self.options = kwargs

    # -- lifecycle -------------------------------------------------------------
    def load(self):
        """Allocate weights / warm up (called once per version on load)."""

    def unload(self):
        """Release resources."""

    # -- metadata ----------------------------------------------------------------
    def config(self):
        cfg = mc.ModelConfig(name=self.name, platform=self.platform, backend=self.backend)
        cfg.max_batch_size = self.max_batch_size
        for t in self.inputs:
            i = cfg.input.add(name=t.name, data_type=cfg_dtype(t.datatype), dims=t.dims)
            if t.fmt == "NCHW":
                i.format = mc.ModelInput.FORMAT_NCHW
            elif t.fmt == "NHWC":
                i.format = mc.ModelInput.FORMAT_NHWC
            if t.optional:
                i.optional = True
        for t in self.outputs:
            o = cfg.output.add(name=t.name, data_type=cfg_dtype(t.datatype), dims=t.dims)
            if t.label_filename:
                o.label_filename = t.label_filename
        if self.dynamic_batching is not None:
            db = cfg.dynamic_batching
            db.preferred_batch_size.extend(self.dynamic_batching.get("preferred", []))
            db.max_queue_delay_microseconds = self.dynamic_batching.get("max_queue_delay_us", 0)
        if self.sequence_batching:
            sb = cfg.sequence_batching
            sb.max_sequence_idle_microseconds = 5000000
        if self.ensemble_steps:
            for model_name, imap, omap in self.ensemble_steps:
                st = cfg.ensemble_scheduling.step.add(model_name=model_name, model_version=-1)
                for k, v in imap.items():
                    st.input_map[k] = v
                for k, v in omap.items():
                    st.output_map[k] = v
        if self.decoupled:
            cfg.model_transaction_policy.decoupled = True
        g = cfg.instance_group.add(
            name=self.name, count=self.instance_count, kind=getattr(mc.ModelInstanceGroup, self.instance_kind)
        )
        g.gpus.extend(self.gpus)
        cfg.version_policy.latest.num_versions = len(self.versions)
        return cfg

    def metadata_tensors(self):
        """(inputs, outputs) lists of (name, datatype, shape) for metadata."""
        prefix = [-1] if self.max_batch_size > 0 else []
        ins = [(t.name, t.datatype, prefix + t.dims) for t in self.inputs]
        outs = [(t.name, t.datatype, prefix + t.dims) for t in self.outputs]
        return ins, outs

    # -- execution -----------------------------------------------------------------
    def execute(self, requests):
        raise NotImplementedError

    def execute_decoupled(self, request, emit):
        raise NotImplementedError

    # -- helpers -------------------------------------------------------------------
    def validate(self, request):
        """Check inputs against the config (names, dtypes, shapes)."""
        by_name = {t.name: t for t in self.inputs}
        seen = set()
        for t in request.inputs:
            spec = by_name.get(t.name)
            if spec is None:
                raise ServerError(
                    "unexpected inference input '%s' for model '%s'" % (t.name, self.name)
                )
            if t.datatype != spec.datatype:
                raise ServerError(
                    "inference input '%s' data-type is '%s', but model '%s' expects '%s'"
                    % (t.name, t.datatype, self.name, spec.datatype)
                )
            dims = list(t.shape)
            if self.max_batch_size > 0:
                if not dims:
                    raise ServerError("input '%s' is missing the batch dimension" % t.name)
                if dims[0] > self.max_batch_size:
                    raise ServerError(
                        "inference request batch-size must be <= %d for '%s'"
                        % (self.max_batch_size, self.name)
                    )
                dims = dims[1:]
            if len(dims) != len(spec.dims) or any(
                s != -1 and s != d for s, d in zip(spec.dims, dims)
            ):
                raise ServerError(
                    "unexpected shape for input '%s' for model '%s'. Expected %s, got %s"
                    % (t.name, self.name, spec.dims, list(t.shape))
                )
            seen.add(t.name)
        for spec in self.inputs:
            if spec.name not in seen and not spec.optional:
                raise ServerError(
                    "expected %d inputs but got %d inputs for model '%s'"
                    % (len(self.inputs), len(request.inputs), self.name)
                )

    def out(self, name, arr, datatype=None):
        spec = next((o for o in self.outputs if o.name == name), None)
        dt = datatype or (spec.datatype if spec else None)
        return OutputTensor(name=name, datatype=dt, shape=list(np.shape(arr)), data=arr)
