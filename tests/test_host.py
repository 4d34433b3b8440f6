"""Host-side logic of the product package: packing, keys, RNG contract (no GPU)."""
import numpy as np
import pytest

from oracle import spec
from yacht_amd import rng
from yacht_amd.state import (PlayerState, YachtState, decode_bid_action, encode_bid_action, pack, string_representation,
                             unpack)


def test_pack_matches_spec_and_roundtrips(golden):
    W = golden("states.npz")["states"]
    strs = set()
    for w in W[:2000]:
        s = unpack(w)
        assert [int(x) for x in pack(s)] == [int(x) for x in w]
        d = spec.unpack_words(w)
        assert d["p1"]["carry"] == s.p1.carry and d["p2"]["cat_scores"] == s.p2.cat_scores
        strs.add(string_representation(s))
    assert len(strs) == 2000  # injective on stringRepresentation's fields


def test_pack_rejects_unrepresentable_states():
    with pytest.raises(ValueError):
        pack(YachtState(p1=PlayerState(carry=[1] * 11)))
    with pytest.raises(ValueError):
        pack(YachtState(p1_bid=("A", 250)))
    with pytest.raises(ValueError):
        pack(YachtState(p2=PlayerState(cat_scores=[500] + [0] * 11)))


def test_string_representation_format():
    s = YachtState(round_no=3, phase=1, rollA=[1, 2, 3, 4, 5], rollB=[6, 6, 6, 6, 6], p1_bid=("B", 1500),
                   p1=PlayerState(carry=[1, 2], used_mask=5, bid_score=-1500))
    assert string_representation(s).startswith("r3|ph1|A12345|B66666|p1bB1500|p2b-|p1c12|p2c|p1u5|p2u0|")


def test_bid_codec():
    for a in range(202):
        t, amt = decode_bid_action(a)
        assert encode_bid_action(t, amt) == a


def test_host_rng_is_the_spec_stream():
    for seed, env in ((0, 0), (123456789123, 77), (2**64 - 1, 2**32 - 1)):
        assert [rng.draw64(seed, env, c) for c in range(40)] == [spec.draw64(seed, env, c) for c in range(40)]
