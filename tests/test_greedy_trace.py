"""Config C1 (BASELINE.json configs[0]): the reference's own main.py loop with greedy
agents on one env, recorded by tests/golden/gen_greedy.py (greedy.npz: actions, executed
actions, collision pairs and canonical states per step; greedy.json: env.get_repr() after
reset and every step, termination_info, all_subtasks).  The engine replays the recorded
action dicts; the shim must reproduce the reference's state reprs character for character.

The greedy actions themselves come from the reference planners (recipe planner, greedy
delegation, BRTDP navigation), which are outside this engine's scope; what is
pinned is everything the env does with them.  Subtask lists are also checked against
tests/golden/subtasks.json (gen_subtasks.py, every builtin level, five hash seeds)."""
import json
import os
import types

import numpy as np
import pytest

import oc_testlib as tl
from gym_cooking_amd import capi, envs, levels, recipes

from oracle import oracle


def _meta():
    with open(os.path.join(tl.GOLDEN, "greedy.json")) as f:
        return json.load(f)


def _env_repr(agents, world):
    """OvercookedEnvironment.get_repr (overcooked_environment.py:50-62) of host views."""
    return repr(world.get_repr() + tuple(a.get_repr() for a in agents))


def _unordered(subtask: str) -> str:
    name, args = subtask[:-1].split("(", 1)
    return "%s(%s)" % (name, ", ".join(sorted(args.split(", "))))


def test_fixture_shape():
    fx, meta = tl.load_fixture("greedy.npz"), _meta()
    assert meta["episodes"][0]["level"] == "open-divider_salad" and meta["episodes"][0]["A"] == 2  # C1
    for e, ep in enumerate(meta["episodes"]):
        assert int(fx["ep_T"][e]) == ep["T"] and len(meta["reprs"][e]) == ep["T"] + 1


def test_all_subtasks_match_reference():
    """recipes.all_subtasks == the reference's env.all_subtasks (sorted) for every builtin
    level under PYTHONHASHSEED=0, and is one of the variants every hash seed produced."""
    with open(os.path.join(tl.GOLDEN, "subtasks.json")) as f:
        fx = json.load(f)["variants"]
    assert set(fx) == set(levels.BUILTIN_LEVELS)
    for name, variants in fx.items():
        ours = sorted(str(s) for s in recipes.all_subtasks(levels.BUILTIN_LEVELS[name]))
        seed0 = [v["sorted"] for v in variants if "0" in v["seeds"]]
        assert ours == seed0[0], name
        # the variants differ only in which of Merge(a, b) / Merge(b, a) is kept
        canon = {tuple(sorted(_unordered(s) for s in v["sorted"])) for v in variants}
        assert len(canon) == 1, name
    for ep in _meta()["episodes"]:
        ours = sorted(str(s) for s in recipes.all_subtasks(levels.load_level(ep["level"])))
        assert ours == ep["all_subtasks"], ep["level"]


def test_parallel_action_choice_matches_reference_set_order():
    """Of two actions with one transition the reference's generate_graph keeps the one its
    recipe.actions set iterates last (stripsworld.py:50-70); recipes._HASH0_KEPT must be that
    choice in the PYTHONHASHSEED=0 orders tests/golden/gen_recipe_order.py recorded."""
    with open(os.path.join(tl.GOLDEN, "recipe_order.json")) as f:
        orders = json.load(f)["orders"]
    for recipe in ("SimpleTomato", "SimpleLettuce", "Salad", "OnionSalad"):
        order = orders["0"][recipe]
        acts, _ = recipes.recipe_actions(recipe)
        assert sorted(order) == sorted(str(a) for a in acts), recipe
        kept = set()
        for a in acts:
            for b in acts:
                if a is not b and a.name == b.name == "Merge" and sorted(a.pre) == sorted(b.pre) and \
                        sorted(a.post_add) == sorted(b.post_add):
                    kept.add(max(str(a), str(b), key=order.index))
        assert kept == set(recipes._HASH0_KEPT.get(recipe, ())), recipe
    # other seeds keep other members of the same pairs (the variants subtasks.json records)
    assert any(orders[s]["OnionSalad"].index("Merge(Onion, Tomato)") < orders[s]["OnionSalad"].index(
        "Merge(Tomato, Onion)") for s in orders)


def test_subtask_masks_match_planner_table():
    """subtask_masks == the oc_subtask masks nav_utils.get_subtask_obj implies (the Salad
    table the rollout fixtures were recorded with, tests/golden/gen_rollout.py)."""
    m = {str(s): recipes.subtask_masks(s) for s in recipes.all_subtasks(levels.load_level("open-divider_salad"))}
    assert m["Chop(Tomato)"] == (1, (0x01, 0), 0x11)
    assert m["Chop(Lettuce)"] == (1, (0x02, 0), 0x22)
    assert m["Merge(Tomato, Lettuce)"] == (2, (0x11, 0x22), 0x33)
    assert m["Merge(Lettuce, Plate)"] == (2, (0x22, 0x08), 0x2A)
    assert m["Merge(Lettuce, Plate-Tomato)"] == (2, (0x22, 0x19), 0x3B)
    assert m["Merge(Lettuce-Tomato, Plate)"] == (2, (0x33, 0x08), 0x3B)
    assert m["Deliver(Lettuce-Plate-Tomato)"] == (3, (0x3B, 0), 0x3B)
    assert recipes.subtask_masks(None) == (0, (0, 0), 0)


def test_oracle_views_reproduce_reference_reprs():
    """Oracle replay of every greedy episode; the shim's host views (with the episode's
    group-name history) print exactly the reference's env.get_repr() at every step."""
    fx, meta = tl.load_fixture("greedy.npz"), _meta()
    for e, ep in enumerate(meta["episodes"]):
        lv = levels.load_level(ep["level"])
        A = ep["A"]
        ob = oracle.OracleBatch(lv, A, 100, 1)
        s, s2 = ob.new_state(), ob.new_state()
        ob.reset(s)
        names = set()
        for step in range(ep["T"] + 1):
            ev = tl.env_view(s, A, ob.K, ob.pitch, 1)[:, 0]
            agents, world, t, _ = envs.build_views(lv, A, ob.K, ev, group_names=sorted(names))
            names |= {it.name for it in world.items}
            assert _env_repr(agents, world) == meta["reprs"][e][step], (ep["level"], ep["seed"], step)
            if step == ep["T"]:
                break
            act = ob.new_actions()
            act.reshape(A, ob.pitch)[:, 0] = fx["act"][fx["ep_act_off"][e] + step][:A]
            ob.step(s, s2, act)
            s, s2 = s2, s


@pytest.mark.gpu
def test_shim_replays_greedy_episodes():
    """The gym shim on the GPU, driven like main.py:85-117 with the recorded action dicts:
    reprs, reward, done, termination_info, collisions and executed actions all match."""
    from gym_cooking_amd.envs import OvercookedEnvironment
    fx, meta = tl.load_fixture("greedy.npz"), _meta()
    for e, ep in enumerate(meta["episodes"]):
        A = ep["A"]
        arg = types.SimpleNamespace(level=ep["level"], num_agents=A, max_num_timesteps=100, max_num_subtasks=14,
                                    seed=ep["seed"], model1="greedy", model2="greedy", model3=None, model4=None,
                                    record=False, with_image_obs=False)
        env = OvercookedEnvironment(arg)
        obs = env.reset()
        assert repr(obs.get_repr()) == meta["reprs"][e][0]
        assert sorted(str(s) for s in env.all_subtasks) == ep["all_subtasks"]
        step = 0
        while not env.done():
            codes = fx["act"][fx["ep_act_off"][e] + step][:A]
            ad = {"agent-%d" % (a + 1): levels.ACTIONS[int(codes[a])] for a in range(A)}
            obs, reward, done, info = env.step(ad)
            step += 1
            assert repr(obs.get_repr()) == meta["reprs"][e][step], (ep["level"], step)
            fl = int(fx["flags"][fx["ep_state_off"][e] + step])
            assert done == bool(fl & 1) and reward == (1 if fl & 2 else 0)
            ex = [levels.ACTION_CODE[env.agent_actions["agent-%d" % (a + 1)]] for a in range(A)]
            assert ex == [int(v) for v in fx["exe"][fx["ep_act_off"][e] + step - 1][:A]]
        assert step == ep["T"]
        assert env.termination_info == ep["termination_info"] and env.successful == ep["successful"]
