"""Short names of the chain render's schedule fields (include/rtx.h
rtx_schedule) for the tuning tools: "a1=1.5,coop=32" -> set_schedule kwargs."""

SHORT = {"a1": "tier1_bar", "a1s": "tier1_bar_small", "a1l": "tier1_bar_low", "a2s": "tier2_bar_small",
         "a2m": "tier2_bar_medium", "a2": "tier2_bar", "rho": "small_share", "rhol": "low_share", "rho2": "medium_share",
         "prio": "hot_fraction", "occs": "occupancy_small", "occl": "occupancy_low", "occn": "occupancy_normal",
         "coop": "tail_coop_max", "coopL": "tail_coop_max_large", "p1": "tier1_priority", "trs": "trace_small", "trl": "trace_low",
         "trm": "trace_medium", "trL": "trace_large", "prs": "promote_small", "prl": "promote_low",
         "prm": "promote_medium", "prL": "promote_large", "prB": "promote_big_scene", "p2": "tier2_priority", "ph": "hot_priority",
         "chunk": "refill_chunk", "tg": "trace_group", "tsolo": "trace_solo_bar",
         "capS": "prepass_cap_split", "pb1": "prio_bar1", "pb2": "prio_bar2", "pb3": "prio_bar3"}


def schedule_of(setting):
    fields = {}
    for kv in filter(None, setting.split(",")):
        k, v = kv.split("=")
        k = SHORT.get(k.strip(), k.strip())
        fields[k] = int(v) if k.startswith("tail_coop_max") or k.endswith("priority") or k in ("refill_chunk", "trace_group", "prepass_cap_split") else float(v)
    return fields
