"""GEMM tuning database (ops.TUNE_DB): round trip, tile-table digest, the
exclusion filter, and that a shipped database matches this tree's tables."""
import json
import os

import pytest

from splatt3r_amd import ops


@pytest.fixture
def fresh_db_state(monkeypatch):
    monkeypatch.setattr(ops, "_TUNE_CACHE", {})
    monkeypatch.setattr(ops, "_DB_STATE", {"loaded": set(), "entries": {}})
    monkeypatch.setattr(ops, "TUNE_COLD", True)
    yield


def _reload(monkeypatch, path):
    monkeypatch.setattr(ops, "TUNE_DB", str(path))
    monkeypatch.setattr(ops, "_TUNE_CACHE", {})
    monkeypatch.setattr(ops, "_DB_STATE", {"loaded": set(), "entries": {}})
    ops._db_load()
    return dict(ops._TUNE_CACHE)


def test_round_trip_keeps_keys_and_like(tmp_path, monkeypatch, fresh_db_state):
    k1 = ("gfx950", 768, 1024, 4096, 1, True, False, None)
    k2 = ("gfx950", 6144, 1024, 4096, 1, True, False, (4, 1))
    ops._TUNE_CACHE.update({k1: (4, 1), k2: (36, 1)})
    p = tmp_path / "db.json"
    ops.save_tune_db(str(p))
    assert _reload(monkeypatch, p) == {k1: (4, 1), k2: (36, 1)}


def test_changed_tile_tables_void_the_file(tmp_path, monkeypatch, fresh_db_state):
    p = tmp_path / "db.json"
    p.write_text(json.dumps({"digest": "not-this-tree", "entries": [[[1, 2, 3, None], [4, 1]]]}))
    assert _reload(monkeypatch, p) == {}


def test_excluded_and_unknown_tiles_are_retuned(tmp_path, monkeypatch, fresh_db_state):
    p = tmp_path / "db.json"
    ents = [[[1, 1, 1, None], [51, 1]], [[2, 2, 2, None], [999, 1]], [[3, 3, 3, None], [32, 2]]]
    p.write_text(json.dumps({"digest": ops._db_digest(), "abi": ops._KERNEL_ABI, "entries": ents}))
    monkeypatch.setattr(ops, "_EXCLUDED", set(ops._HALO))
    assert _reload(monkeypatch, p) == {("gfx950", 3, 3, 3, None): (32, 2)}


def test_warm_tuning_policy_ignores_the_cold_database(tmp_path, monkeypatch, fresh_db_state):
    p = tmp_path / "db.json"
    p.write_text(json.dumps({"digest": ops._db_digest(), "entries": [[[3, 3, 3, None], [32, 1]]]}))
    monkeypatch.setattr(ops, "TUNE_COLD", False)
    assert _reload(monkeypatch, p) == {}


def test_shipped_database_matches_this_tree():
    path = os.path.join(os.path.dirname(ops.__file__), "tune_gfx950.json")
    if not os.path.isfile(path):
        pytest.skip("no shipped tuning database")
    with open(path) as f:
        db = json.load(f)
    assert db["digest"] == ops._db_digest()
    for k, v in db["entries"]:
        assert v[0] == 0 or v[0] in ops._TILE_SHAPES
        if k[-1] is not None and v[0] and k[-1][0]:
            # a batch-invariant plan's choice is in the class of its like
            kk = k[2]
            assert ops.reduction_class(kk, *v) == ops.reduction_class(kk, *k[-1])


def _reload_dev(monkeypatch, path, arch):
    monkeypatch.setattr(ops, "_device_arch", lambda dev: arch)
    monkeypatch.setattr(ops, "TUNE_DB", str(path))
    monkeypatch.setattr(ops, "_TUNE_CACHE", {})
    monkeypatch.setattr(ops, "_DB_STATE", {"loaded": set(), "entries": {}})
    ops._db_load("cuda:0")
    return dict(ops._TUNE_CACHE)


def test_foreign_arch_voids_the_file(tmp_path, monkeypatch, fresh_db_state):
    p = tmp_path / "db.json"
    ents = [[[3, 3, 3, None], [32, 1]]]
    p.write_text(json.dumps({"digest": ops._db_digest(), "abi": ops._KERNEL_ABI,
                             "arch": "gfx950", "entries": ents}))
    assert _reload_dev(monkeypatch, p, "gfx942") == {}
    assert _reload_dev(monkeypatch, p, "gfx950") == {("gfx950", 3, 3, 3, None): (32, 1)}


def test_other_kernel_abi_voids_the_file(tmp_path, monkeypatch, fresh_db_state):
    p = tmp_path / "db.json"
    ents = [[[3, 3, 3, None], [32, 1]]]
    p.write_text(json.dumps({"digest": ops._db_digest(), "abi": "0" * 16,
                             "arch": "gfx950", "entries": ents}))
    assert _reload_dev(monkeypatch, p, "gfx950") == {}


def test_save_records_the_tuned_target(tmp_path, monkeypatch, fresh_db_state):
    """save_tune_db labels the file with the gfx target the choices were
    tuned on, and a file tuned elsewhere is not loaded here."""
    ops._TUNE_CACHE.update({("gfx942", 3, 3, 3, None): (32, 1)})
    p = tmp_path / "db.json"
    ops.save_tune_db(str(p))
    assert json.loads(p.read_text())["arch"] == "gfx942"
    assert _reload_dev(monkeypatch, p, "gfx950") == {}
    assert _reload_dev(monkeypatch, p, "gfx942") == {("gfx942", 3, 3, 3, None): (32, 1)}
    ops._TUNE_CACHE.update({("gfx950", 3, 3, 3, None): (5, 1)})
    with pytest.raises(ValueError):
        ops.save_tune_db(str(p))


def test_kernel_abi_is_a_digest_of_the_gemm_sources():
    """The database's kernel-ABI stamp follows the GEMM sources: it is a
    source digest, not a hand-bumped constant."""
    assert ops._KERNEL_ABI == ops._kernel_abi() != "unknown"
    assert len(ops._KERNEL_ABI) == 16
    with open(os.path.join(os.path.dirname(ops.__file__), "tune_gfx950.json")) as f:
        assert json.load(f)["abi"] == ops._KERNEL_ABI, "re-tune: the GEMM sources changed"
