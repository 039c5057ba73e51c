"""oracle -- TEST INFRASTRUCTURE ONLY.

CPU restatement of the DQN learn-step hot path of youcefMehamlia/Multimodal-DRL-RMC
(`dqn.agent.Agent.learn()`, `dqn.network`, `dqn.replay_memory`, `dqn.utils.sum_tree`).
It is the *checker* for the MI355X engine in ``multimodal-drl-rmc_amd/``: only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import it, and never as the thing measured or shipped.  The product path has no
CPU fallback and never routes through this package.

Pinning (see DESIGN.md "Oracle"):
  * ``pyrandom.c`` (MT19937 / random.sample / numpy legacy uniform) is checked
    against CPython's ``random.sample`` and numpy's ``RandomState`` directly, and
    against ``tests/golden/*.npz`` generated from the reference itself
    (``tests/golden/make_golden.py`` imports /root/reference in the build
    container only).
  * ``ref.py`` (networks, learn steps, Adam, soft update, replay, SumTree) is
    checked against the same golden fixtures: sampled indices bit-exact, Q/loss/
    weights within 1e-5.
"""
