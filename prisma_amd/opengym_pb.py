"""The ns3-gym wire messages (package ``ns3opengym``; the reference's
prisma/ns3_model/messages.proto:1-123) as protobuf classes built at import time from a
descriptor, since ``protoc`` is not installed.  Field numbers, types and names follow
the reference interface so the bytes are those its ``messages_pb2`` produces and parses.
Only the messages the packet-routing protocol exchanges are declared (Discrete and Box
spaces / containers; no Tuple / Dict)."""
from __future__ import annotations

from google.protobuf import any_pb2, descriptor_pb2, descriptor_pool
from google.protobuf import message_factory

F = descriptor_pb2.FieldDescriptorProto


def _file() -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto(name="prisma_amd/ns3opengym_messages.proto", package="ns3opengym",
                                            syntax="proto3")
    fd.dependency.append("google/protobuf/any.proto")

    def enum(name, values, parent=None):
        e = (parent.enum_type if parent is not None else fd.enum_type).add(name=name)
        for i, v in enumerate(values):
            e.value.add(name=v, number=i)

    enum("MsgType", ["Unknown", "Init", "ActionSpace", "ObservationSpace", "IsGameOver", "Observation", "Reward",
                     "ExtraInfo", "Action", "StopEnv"])
    enum("SpaceType", ["NoSpaceType", "Discrete", "Box", "Tuple", "Dict"])
    enum("Dtype", ["NoDType", "INT", "UINT", "FLOAT", "DOUBLE"])

    def msg(name, fields):
        m = fd.message_type.add(name=name)
        for num, fname, ftype, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=ftype, label=label or F.LABEL_OPTIONAL)
            if tname:
                f.type_name = tname
        return m

    R, O = F.LABEL_REPEATED, None
    msg("SpaceDescription", [(1, "type", F.TYPE_ENUM, O, ".ns3opengym.SpaceType"),
                             (2, "space", F.TYPE_MESSAGE, O, ".google.protobuf.Any"),
                             (3, "name", F.TYPE_STRING, O, None)])
    msg("DiscreteSpace", [(1, "n", F.TYPE_INT32, O, None)])
    msg("BoxSpace", [(1, "low", F.TYPE_FLOAT, O, None), (2, "high", F.TYPE_FLOAT, O, None),
                     (3, "dtype", F.TYPE_ENUM, O, ".ns3opengym.Dtype"), (4, "shape", F.TYPE_UINT32, R, None)])
    msg("DataContainer", [(1, "type", F.TYPE_ENUM, O, ".ns3opengym.SpaceType"),
                          (2, "data", F.TYPE_MESSAGE, O, ".google.protobuf.Any"),
                          (3, "name", F.TYPE_STRING, O, None)])
    msg("DiscreteDataContainer", [(1, "data", F.TYPE_INT32, O, None)])
    msg("BoxDataContainer", [(1, "dtype", F.TYPE_ENUM, O, ".ns3opengym.Dtype"), (2, "shape", F.TYPE_UINT32, R, None),
                             (3, "intData", F.TYPE_INT32, R, None), (4, "uintData", F.TYPE_UINT32, R, None),
                             (5, "floatData", F.TYPE_FLOAT, R, None), (6, "doubleData", F.TYPE_DOUBLE, R, None)])
    msg("SimInitMsg", [(1, "simProcessId", F.TYPE_UINT64, O, None), (2, "wafShellProcessId", F.TYPE_UINT64, O, None),
                       (3, "obsSpace", F.TYPE_MESSAGE, O, ".ns3opengym.SpaceDescription"),
                       (4, "actSpace", F.TYPE_MESSAGE, O, ".ns3opengym.SpaceDescription")])
    msg("SimInitAck", [(1, "done", F.TYPE_BOOL, O, None), (2, "stopSimReq", F.TYPE_BOOL, O, None)])
    st = msg("EnvStateMsg", [(1, "obsData", F.TYPE_MESSAGE, O, ".ns3opengym.DataContainer"),
                             (2, "reward", F.TYPE_FLOAT, O, None), (3, "isGameOver", F.TYPE_BOOL, O, None),
                             (4, "reason", F.TYPE_ENUM, O, ".ns3opengym.EnvStateMsg.Reason"),
                             (5, "info", F.TYPE_STRING, O, None)])
    enum("Reason", ["SimulationEnd", "GameOver"], parent=st)
    msg("EnvActMsg", [(1, "actData", F.TYPE_MESSAGE, O, ".ns3opengym.DataContainer"),
                      (2, "stopSimReq", F.TYPE_BOOL, O, None)])
    return fd


_pool = descriptor_pool.DescriptorPool()
_pool.AddSerializedFile(any_pb2.DESCRIPTOR.serialized_pb)
_fdesc = _pool.AddSerializedFile(_file().SerializeToString())
_classes = message_factory.GetMessages([_file()], pool=_pool)

SpaceDescription = _classes["ns3opengym.SpaceDescription"]
DiscreteSpace = _classes["ns3opengym.DiscreteSpace"]
BoxSpace = _classes["ns3opengym.BoxSpace"]
DataContainer = _classes["ns3opengym.DataContainer"]
DiscreteDataContainer = _classes["ns3opengym.DiscreteDataContainer"]
BoxDataContainer = _classes["ns3opengym.BoxDataContainer"]
SimInitMsg = _classes["ns3opengym.SimInitMsg"]
SimInitAck = _classes["ns3opengym.SimInitAck"]
EnvStateMsg = _classes["ns3opengym.EnvStateMsg"]
EnvActMsg = _classes["ns3opengym.EnvActMsg"]

# enum values (messages.proto:7-34, 112-115)
Discrete, Box = 1, 2
INT, UINT, FLOAT, DOUBLE = 1, 2, 3, 4
SimulationEnd, GameOver = 0, 1
