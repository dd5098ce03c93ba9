"""Wire schema of the codec payloads: NamedTensor / MetadataProto.

Mirrors openfl/protocols/base.proto:11-25 field-for-field (numbers and types,
so bytes interoperate with the reference's generated base_pb2) and
construct_named_tensor (openfl/protocols/utils.py:101-147).  The message
classes are built at run time from a FileDescriptorProto (this image has no
protoc / grpc_tools).
"""
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

_F = descriptor_pb2.FieldDescriptorProto


def _build():
    fdp = descriptor_pb2.FileDescriptorProto(name="openfl_amd/wire/base.proto", package="openfl_amd.wire",
                                             syntax="proto3")
    md = fdp.message_type.add(name="MetadataProto")
    entry = md.nested_type.add(name="IntToFloatEntry")
    entry.options.map_entry = True
    entry.field.add(name="key", number=1, type=_F.TYPE_INT32, label=_F.LABEL_OPTIONAL)
    entry.field.add(name="value", number=2, type=_F.TYPE_FLOAT, label=_F.LABEL_OPTIONAL)
    md.field.add(name="int_to_float", number=1, type=_F.TYPE_MESSAGE, label=_F.LABEL_REPEATED,
                 type_name=".openfl_amd.wire.MetadataProto.IntToFloatEntry")
    md.field.add(name="int_list", number=2, type=_F.TYPE_INT32, label=_F.LABEL_REPEATED)
    md.field.add(name="bool_list", number=3, type=_F.TYPE_BOOL, label=_F.LABEL_REPEATED)
    nt = fdp.message_type.add(name="NamedTensor")
    nt.field.add(name="name", number=1, type=_F.TYPE_STRING, label=_F.LABEL_OPTIONAL)
    nt.field.add(name="round_number", number=2, type=_F.TYPE_INT32, label=_F.LABEL_OPTIONAL)
    nt.field.add(name="lossless", number=3, type=_F.TYPE_BOOL, label=_F.LABEL_OPTIONAL)
    nt.field.add(name="report", number=4, type=_F.TYPE_BOOL, label=_F.LABEL_OPTIONAL)
    nt.field.add(name="tags", number=5, type=_F.TYPE_STRING, label=_F.LABEL_REPEATED)
    nt.field.add(name="transformer_metadata", number=6, type=_F.TYPE_MESSAGE, label=_F.LABEL_REPEATED,
                 type_name=".openfl_amd.wire.MetadataProto")
    nt.field.add(name="data_bytes", number=7, type=_F.TYPE_BYTES, label=_F.LABEL_OPTIONAL)
    mp = fdp.message_type.add(name="ModelProto")
    mp.field.add(name="tensors", number=1, type=_F.TYPE_MESSAGE, label=_F.LABEL_REPEATED,
                 type_name=".openfl_amd.wire.NamedTensor")
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    get = message_factory.GetMessageClass
    return (get(pool.FindMessageTypeByName("openfl_amd.wire.MetadataProto")),
            get(pool.FindMessageTypeByName("openfl_amd.wire.NamedTensor")),
            get(pool.FindMessageTypeByName("openfl_amd.wire.ModelProto")))


MetadataProto, NamedTensor, ModelProto = _build()


def construct_named_tensor(tensor_key, nparray, transformer_metadata, lossless):
    """utils.py:101-147: metadata dicts -> MetadataProto list; data_bytes = payload."""
    protos = []
    for m in transformer_metadata:
        protos.append(MetadataProto(int_to_float=m.get("int_to_float") or {},
                                    int_list=m.get("int_list") or [],
                                    bool_list=m.get("bool_list") or []))
    name, origin, round_number, report, tags = tensor_key
    return NamedTensor(name=name, round_number=round_number, lossless=lossless, report=report, tags=tags,
                       transformer_metadata=protos, data_bytes=nparray)


def transformer_metadata_of(named_tensor):
    """The list-of-dicts a receiver hands to pipeline.backward
    (collaborator.py:552-559, aggregator.py:710-717): protobuf containers."""
    return [{"int_to_float": p.int_to_float, "int_list": p.int_list, "bool_list": p.bool_list}
            for p in named_tensor.transformer_metadata]
