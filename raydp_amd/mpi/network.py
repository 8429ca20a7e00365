"""gRPC plumbing for the MPI job protocol without generated code.

The message classes are built from a ``FileDescriptorProto`` assembled here (mirrors
``network.proto`` next to this file; reference: ``python/raydp/mpi/network/network.proto``
and its generated ``network_pb2*.py``). Services are registered with gRPC's generic handler
API and called through plain ``unary_unary`` callables, so no ``grpc_tools`` step exists.
"""
from typing import Callable, Dict, Tuple

import grpc
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

from raydp_amd.mpi.constants import MAX_MESSAGE_LENGTH

_PKG = "raydp.mpi"
_T = descriptor_pb2.FieldDescriptorProto
_FIELDS = {
    "RegisterWorkerRequest": [("job_id", 1, _T.TYPE_STRING, False), ("world_rank", 2, _T.TYPE_INT32, False)],
    "RegisterWorkerReply": [("node_addresses", 3, _T.TYPE_STRING, True)],
    "RegisterWorkerServiceRequest": [("world_rank", 1, _T.TYPE_INT32, False),
                                     ("worker_ip", 2, _T.TYPE_STRING, False),
                                     ("worker_port", 3, _T.TYPE_INT32, False)],
    "RegisterWorkerServiceReply": [("ray_address", 1, _T.TYPE_STRING, False),
                                   ("redis_password", 2, _T.TYPE_STRING, False)],
    "Function": [("func_id", 1, _T.TYPE_INT32, False), ("func", 2, _T.TYPE_BYTES, False)],
    "FunctionResult": [("world_rank", 1, _T.TYPE_INT32, False), ("func_id", 2, _T.TYPE_INT32, False),
                       ("result", 3, _T.TYPE_BYTES, False)],
    "Empty": [],
}
# service -> method -> (request, response)
SERVICES: Dict[str, Dict[str, Tuple[str, str]]] = {
    "DriverService": {
        "RegisterWorker": ("RegisterWorkerRequest", "RegisterWorkerReply"),
        "RegisterWorkerService": ("RegisterWorkerServiceRequest", "RegisterWorkerServiceReply"),
        "RegisterFuncResult": ("FunctionResult", "Empty"),
    },
    "WorkerService": {
        "RunFunction": ("Function", "Empty"),
        "Stop": ("Empty", "Empty"),
    },
}


def _build():
    fdp = descriptor_pb2.FileDescriptorProto(name="raydp_mpi_network.proto", package=_PKG, syntax="proto3")
    for name, fields in _FIELDS.items():
        m = fdp.message_type.add(name=name)
        for fname, num, typ, rep in fields:
            m.field.add(name=fname, number=num, type=typ,
                        label=_T.LABEL_REPEATED if rep else _T.LABEL_OPTIONAL)
    for sname, methods in SERVICES.items():
        s = fdp.service.add(name=sname)
        for mname, (req, resp) in methods.items():
            s.method.add(name=mname, input_type=f".{_PKG}.{req}", output_type=f".{_PKG}.{resp}")
    pool = descriptor_pool.DescriptorPool()
    fd = pool.Add(fdp)
    return {name: message_factory.GetMessageClass(pool.FindMessageTypeByName(f"{_PKG}.{name}"))
            for name in _FIELDS}, fd


messages, FILE_DESCRIPTOR = _build()
RegisterWorkerRequest = messages["RegisterWorkerRequest"]
RegisterWorkerReply = messages["RegisterWorkerReply"]
RegisterWorkerServiceRequest = messages["RegisterWorkerServiceRequest"]
RegisterWorkerServiceReply = messages["RegisterWorkerServiceReply"]
Function = messages["Function"]
FunctionResult = messages["FunctionResult"]
Empty = messages["Empty"]

CHANNEL_OPTIONS = (("grpc.enable_http_proxy", 0),
                   ("grpc.max_send_message_length", MAX_MESSAGE_LENGTH),
                   ("grpc.max_receive_message_length", MAX_MESSAGE_LENGTH))


def add_service(server: grpc.Server, service: str, impl) -> None:
    """Register ``impl.<Method>(request, context)`` for every method of ``service``."""
    handlers = {}
    for mname, (req, resp) in SERVICES[service].items():
        handlers[mname] = grpc.unary_unary_rpc_method_handler(
            getattr(impl, mname), request_deserializer=messages[req].FromString,
            response_serializer=messages[resp].SerializeToString)
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(f"{_PKG}.{service}", handlers),))


class Stub:
    """Client for one service: ``stub.RegisterWorker(msg, timeout=...)``."""

    def __init__(self, channel: grpc.Channel, service: str):
        self._channel = channel
        for mname, (req, resp) in SERVICES[service].items():
            setattr(self, mname, channel.unary_unary(
                f"/{_PKG}.{service}/{mname}", request_serializer=messages[req].SerializeToString,
                response_deserializer=messages[resp].FromString))

    def close(self):
        self._channel.close()


def insecure_channel(address: str, options=None) -> grpc.Channel:
    """Channel with the HTTP proxy disabled (reference: ``mpi/utils.py`` create_insecure_channel)."""
    opts = list(options or ())
    if not any(k == "grpc.enable_http_proxy" for k, _ in opts):
        opts.append(("grpc.enable_http_proxy", 0))
    opts += [o for o in CHANNEL_OPTIONS if o[0] != "grpc.enable_http_proxy"]
    return grpc.insecure_channel(address, opts)


def make_server(max_workers: int = 2) -> grpc.Server:
    from concurrent import futures
    return grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers), options=CHANNEL_OPTIONS)


Handler = Callable
