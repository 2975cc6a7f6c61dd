"""gRPC span server on the gfx950 engine: a wire-compatible drop-in for the reference's
`models/qwen3/server/server.py` (Qwen3LayerServicer.ProcessLayer, :25-54) behind the same
service, method and messages (`models/qwen3/proto/qwen3.proto:5-24`):

    service qwen3.Qwen3Layer { rpc ProcessLayer(LayerRequest) returns (LayerResponse); }
    LayerRequest  { TensorBlob hidden_states, attention_mask, cache_position,
                    cos_embedding, sin_embedding; string session_id; }
    LayerResponse { TensorBlob hidden_states; }     TensorBlob { bytes data; }

The message classes are built at import from a descriptor written here (no generated
`_pb2` module, no protoc), so a stock `RPCQwen3Client` (rpc_client.py:36-57) talks to it
unchanged.

TensorBlob payloads:
  * the reference's form, `torch.save(tensor)` bytes (server.py:16-23, rpc_client.py:27-34),
    is read with `torch.load(..., weights_only=True)`: a tensor-only loader that executes
    nothing from the blob, where the reference's own `torch.load` would unpickle anything;
  * a raw form, RAW_MAGIC + dtype + shape + the tensor's bytes, costs no pickling: a peer
    that sends raw blobs gets raw blobs back (`blob_to_tensor` / `tensor_to_blob`).
The server answers in the format the request's hidden_states used.

hidden_states, cache_position and session_id drive the computation; the causal mask and
(cos, sin) are derived on the device from the positions, and the request's attention_mask /
cos_embedding / sin_embedding, when present, must be the ones the engine derives
(Qwen3Server.send docstring): anything else is refused with INTERNAL, as an exception in the
reference's forward is (server.py:49-50).
"""
from __future__ import annotations

import io
import struct

import numpy as np
import torch

from .qwen3_server import Qwen3Server

RAW_MAGIC = b"IFDRAW01"
_DTYPES = {"float32": torch.float32, "bfloat16": torch.bfloat16, "float16": torch.float16,
           "int64": torch.int64, "int32": torch.int32, "bool": torch.bool}
_CODES = {v: k for k, v in _DTYPES.items()}


# ------------------------------------------------------------------ blob codec
def tensor_to_blob(t: torch.Tensor, raw: bool = False) -> bytes:
    """TensorBlob.data for `t`: torch.save bytes (the reference's format) or the raw form."""
    t = t.detach().cpu().contiguous()
    if not raw:
        buf = io.BytesIO()
        torch.save(t, buf)
        return buf.getvalue()
    name = _CODES[t.dtype].encode()
    head = RAW_MAGIC + struct.pack("<B", len(name)) + name + struct.pack("<B", t.dim()) + \
        struct.pack(f"<{t.dim()}q", *t.shape)
    if t.dtype == torch.bfloat16:
        body = t.view(torch.int16).numpy().tobytes()
    elif t.dtype == torch.bool:
        body = t.to(torch.uint8).numpy().tobytes()
    else:
        body = t.numpy().tobytes()
    return head + body


def blob_is_raw(data: bytes) -> bool:
    return data[:len(RAW_MAGIC)] == RAW_MAGIC


def blob_to_tensor(data: bytes) -> torch.Tensor:
    """Inverse of tensor_to_blob for either format (torch.save blobs load weights-only)."""
    if not blob_is_raw(data):
        return torch.load(io.BytesIO(data), map_location="cpu", weights_only=True)
    o = len(RAW_MAGIC)
    n = data[o]
    name = data[o + 1:o + 1 + n].decode()
    o += 1 + n
    nd = data[o]
    shape = struct.unpack(f"<{nd}q", data[o + 1:o + 1 + 8 * nd])
    body = data[o + 1 + 8 * nd:]
    dt = _DTYPES[name]
    if dt == torch.bfloat16:
        return torch.from_numpy(np.frombuffer(body, dtype=np.int16).copy()).view(torch.bfloat16).reshape(shape)
    if dt == torch.bool:
        return torch.from_numpy(np.frombuffer(body, dtype=np.uint8).copy()).to(torch.bool).reshape(shape)
    npdt = {torch.float32: np.float32, torch.float16: np.float16, torch.int64: np.int64, torch.int32: np.int32}[dt]
    return torch.from_numpy(np.frombuffer(body, dtype=npdt).copy()).reshape(shape)


# ------------------------------------------------------------------ messages (qwen3.proto)
def _build_messages():
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    F = descriptor_pb2.FieldDescriptorProto
    fd = descriptor_pb2.FileDescriptorProto(name="inferd_qwen3.proto", package="qwen3", syntax="proto3")
    blob = fd.message_type.add(name="TensorBlob")
    blob.field.add(name="data", number=1, type=F.TYPE_BYTES, label=F.LABEL_OPTIONAL)
    req = fd.message_type.add(name="LayerRequest")
    for i, n in enumerate(("hidden_states", "attention_mask", "cache_position", "cos_embedding", "sin_embedding"), 1):
        req.field.add(name=n, number=i, type=F.TYPE_MESSAGE, type_name=".qwen3.TensorBlob", label=F.LABEL_OPTIONAL)
    req.field.add(name="session_id", number=6, type=F.TYPE_STRING, label=F.LABEL_OPTIONAL)
    resp = fd.message_type.add(name="LayerResponse")
    resp.field.add(name="hidden_states", number=1, type=F.TYPE_MESSAGE, type_name=".qwen3.TensorBlob",
                   label=F.LABEL_OPTIONAL)
    svc = fd.service.add(name="Qwen3Layer")
    svc.method.add(name="ProcessLayer", input_type=".qwen3.LayerRequest", output_type=".qwen3.LayerResponse")
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    classes = message_factory.GetMessages([fd], pool=pool)
    return classes["qwen3.TensorBlob"], classes["qwen3.LayerRequest"], classes["qwen3.LayerResponse"]


TensorBlob, LayerRequest, LayerResponse = _build_messages()
SERVICE, METHOD = "qwen3.Qwen3Layer", "ProcessLayer"


# ------------------------------------------------------------------ servicer
class Qwen3LayerServicer:
    """server.py:12-54 on the engine: the span is a Qwen3Server(start, end) (inferd_amd)."""

    def __init__(self, start_layer: int, end_layer: int, **server_kw):
        self.server_module = Qwen3Server(start_layer, end_layer, **server_kw)

    def ProcessLayer(self, request, context):
        import grpc
        try:
            hidden = blob_to_tensor(request.hidden_states.data)
            cache_pos = blob_to_tensor(request.cache_position.data) if request.cache_position.data else None
            mask = blob_to_tensor(request.attention_mask.data) if request.attention_mask.data else None
            pe = None
            if request.cos_embedding.data and request.sin_embedding.data:
                pe = (blob_to_tensor(request.cos_embedding.data), blob_to_tensor(request.sin_embedding.data))
        except Exception as e:  # noqa: BLE001 -- mirrors server.py:36-37
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"Failed to deserialize tensors: {e}")
        sid = request.session_id or None          # server.py:39
        try:
            out = self.server_module.send(session_id=sid, hidden_states=hidden.to(torch.bfloat16),
                                          attention_mask=mask, cache_position=cache_pos, position_embeddings=pe)
        except Exception as e:  # noqa: BLE001 -- mirrors server.py:49-50
            context.abort(grpc.StatusCode.INTERNAL, f"Error in model forward: {e}")
        out = out.to(hidden.dtype)
        return LayerResponse(hidden_states=TensorBlob(data=tensor_to_blob(out, raw=blob_is_raw(
            request.hidden_states.data))))


def make_server(servicer: Qwen3LayerServicer, port: int, host: str = "[::]", workers: int = 4):
    """grpc.server with the reference's options (server.py:64-73); returns (server, bound port).
    One worker thread at a time drives the span (the engine serialises per span handle)."""
    import threading
    from concurrent import futures

    import grpc
    lock = threading.Lock()

    def handler(request, context):
        with lock:
            return servicer.ProcessLayer(request, context)

    options = [("grpc.max_receive_message_length", 100 * 1024 * 1024),
               ("grpc.max_send_message_length", 100 * 1024 * 1024)]
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=workers), options=options)
    rpc = grpc.unary_unary_rpc_method_handler(handler, request_deserializer=LayerRequest.FromString,
                                              response_serializer=LayerResponse.SerializeToString)
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(SERVICE, {METHOD: rpc}),))
    bound = server.add_insecure_port(f"{host}:{port}")
    return server, bound


def client_stub(channel):
    """The ProcessLayer callable of a channel (what qwen3_pb2_grpc.Qwen3LayerStub exposes)."""
    return channel.unary_unary(f"/{SERVICE}/{METHOD}", request_serializer=LayerRequest.SerializeToString,
                               response_deserializer=LayerResponse.FromString)


def serve():
    """server.py:57-75: --start_layer --end_layer --port (+ --model / --weights)."""
    import argparse
    p = argparse.ArgumentParser()
    p.add_argument("--start_layer", type=int, required=True)
    p.add_argument("--end_layer", type=int, required=True)
    p.add_argument("--port", type=int, required=True)
    p.add_argument("--model", default="qwen3-0.6b")
    p.add_argument("--weights", default="synthetic:1234",
                   help="synthetic:<seed> or a layer_{idx:02d}.pt pattern (weights-only state dicts)")
    a = p.parse_args()
    server, _ = make_server(Qwen3LayerServicer(a.start_layer, a.end_layer, model=a.model, weights=a.weights),
                            a.port)
    server.start()
    print(f"gRPC server listening on port {a.port}, layers {a.start_layer}-{a.end_layer}")
    server.wait_for_termination()


if __name__ == "__main__":
    serve()
