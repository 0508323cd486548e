"""The reference-pinned KATs (tests/golden/kats.json) on the GPU engine, for every KAT this build applies on
the GPU (gpu_eligible): the same expectations the CPU oracle is pinned against in test_oracle_kats.py."""
import pytest

from tests.kat_runner import EngineBackend, KatRun, all_kats, gpu_eligible

pytestmark = pytest.mark.gpu

KATS = [k for k in all_kats() if gpu_eligible(k)]
REFUSED = [k for k in all_kats() if k.get("gpu") == "refuses"]


def test_gpu_kat_coverage():
    names = {k["name"] for k in KATS}
    assert {"map_put_get_remove", "map_put_if_absent", "A1_replace_if_present_inverts_args", "lock_unlock",
            "election_elect", "group_join", "group_leave", "A7_trylock_timeout_is_silent",
            "lock_delete_then_unlock_commit_closed", "A9_leader_relisten_appended", "map_contains_value", "map_size",
            "map_clear", "map_put_ttl", "map_put_if_absent_ttl", "A5_contains_value_npe_order",
            "A8_timer_deferred_after_commit", "A8_timer_immediate_module_mode", "set_add_remove",
            "set_ttl_size_clear", "group_schedule_fires_on_clock", "dispatch_errors", "queue_offer_poll",
            "queue_add_remove", "queue_null_and_empty_quirks",
            # session close fan-out (close.hip) and the manager control plane (manager.hip)
            "election_next_on_close", "A10_close_publishes_leave_for_non_member", "A11_lock_survives_holder_close",
            "manager_create_concurrency", "manager_get_create_concurrency", "manager_operate_many",
            "manager_get_reuses_instance", "A13_delete_resource_by_instance_id", "A18_multimap_put_never_stores"} <= names
    # every KAT runs through the engine (a KAT marked "gpu": "refuses" would have to fail the batch loudly with
    # CC_ERR_STATE; none is marked any more)
    assert len(KATS) + len(REFUSED) == len(all_kats())
    assert {"A5_contains_value_treeify_resize", "A5_contains_value_string_hash_order", "A5_contains_value_tree_bin_order",
            "A5_tree_bin_put_after_treeify", "A5_tree_bin_remove_and_untreeify", "A12_close_after_tree_bin_removal",
            "A5_tree_bin_leaves_small_window"} <= names
    # none left: a bin that was a tree bin while the table was small is followed past 64 by the map's big model
    assert not REFUSED


@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_kat_on_gpu(kat):
    KatRun(kat, EngineBackend(kat)).run()
