"""Wire schema (openfl/protocols/base.proto:11-25) round trip, on CPU."""
import numpy as np

from openfl_amd import protocols as P


def test_named_tensor_roundtrip():
    md = [{"int_list": [2, 3], "int_to_float": {0: 4242.0, 1: 6.0, 2: 0.125, 3: 8.0}}, {}]
    nt = P.construct_named_tensor(("w", "col1", 3, False, ("trained",)), b"\x01\x02", md, False)
    b = nt.SerializeToString()
    back = P.NamedTensor()
    back.ParseFromString(b)
    assert back.name == "w" and back.round_number == 3 and list(back.tags) == ["trained"]
    assert back.data_bytes == b"\x01\x02"
    got = P.transformer_metadata_of(back)
    assert list(got[0]["int_list"]) == [2, 3]
    assert dict(got[0]["int_to_float"]) == {0: 4242.0, 1: 6.0, 2: 0.125, 3: 8.0}
    assert len(got[1]["int_to_float"]) == 0


def test_int_to_float_is_float32_on_the_wire():
    """map<int32, float>: values are rounded to float32 (quirk 4)."""
    nt = P.construct_named_tensor(("w", "", 0, False, ()), b"", [{"int_to_float": {1: 525336577.0}}], True)
    back = P.NamedTensor()
    back.ParseFromString(nt.SerializeToString())
    assert back.transformer_metadata[0].int_to_float[1] == float(np.float32(525336577.0)) == 525336576.0


def test_field_numbers_match_reference_schema():
    f = {fd.name: (fd.number, fd.type) for fd in P.NamedTensor.DESCRIPTOR.fields}
    assert f["name"][0] == 1 and f["round_number"][0] == 2 and f["lossless"][0] == 3
    assert f["report"][0] == 4 and f["tags"][0] == 5 and f["transformer_metadata"][0] == 6
    assert f["data_bytes"][0] == 7
    m = {fd.name: fd.number for fd in P.MetadataProto.DESCRIPTOR.fields}
    assert m == {"int_to_float": 1, "int_list": 2, "bool_list": 3}
