"""Algorithmic FLOP accounting for the lgx kernels.

The physics figure is an operation count of the *algorithm* lgx_physics_kernel implements
(floating-base CRBA + RNEA, arrowhead Schur solve, two-pass compliant contact), counted once
per env-substep — not the executed instruction count, which replicates the per-env work over
the leg lanes (the PMC cross-check in DESIGN.md §5 reads 42 kFLOP executed at PP=1).
Counting rules: one FLOP per f32 add/sub/mul/div, two per fused multiply-add pair, one per
sqrt / sin / cos; compares, selects and index arithmetic are free.
"""

# elementary blocks
CROSS = 9            # a x b
DOT3 = 5
MATVEC3 = 15
MATMAT3 = 45
QUAT_TO_MAT = 27
AXIS_ANGLE = 2 + 1 + 9 * 3 + 6    # sincos, 1-c, Rodrigues entries
SI_MUL = 15 + CROSS + 3 + CROSS + 3 + 3   # compact spatial inertia x motion vector
CRM = 3 * CROSS + 3
CRF = 3 * CROSS + 3
SI_ADD = 10

# per stage
KIN_PER_JOINT = MATMAT3 + MATVEC3 + 3 + MATVEC3 + AXIS_ANGLE + MATMAT3 + CROSS
BODY_SI = MATMAT3 + 6 * DOT3 + MATVEC3 + 3 + 1 + DOT3 + 3 + 3 * 5 + 3 * 4
RNEA_PER_JOINT = 12 + (CRM + 6 + 6) + (SI_MUL + SI_MUL + CRF + 6)
RNEA_LEG_SUMS = 2 * 6 + 3 * 11
FBASE = CROSS + 6 + 2 * SI_MUL + CRF + 6
CRBA_PER_LEG = 2 * SI_ADD + 3 * SI_MUL + 6 * 11
ACOM = 3 * 10 + SI_ADD
RBCOM = 6 * (6 + 5 + 2)
RB0_PER_LEG = 6 * 7
RL0_PER_LEG = 15 + 3 * (6 + 5 + 3)
DRIVE_PER_JOINT = 10
ARROW_PER_LEG = 30 + 6 * 15 + 15 + 21 * 6 + 6 * 6 + (6 * 6 + 15)
ARROW_PER_ENV = 27 * 4 + 97 + 72          # cross-leg Schur sums + 6x6 Cholesky + 2 solves
STATUS_VL_PER_LEG = 3 * 12
INTEGRATE = 12 * 8 + 6 + 45
# contacts
CAND_TRANSFORM = MATVEC3 + 3 + 4          # point to world, depth
HEIGHT_PLANE = 0
HEIGHT_FIELD = 35                         # triangle of the sampled heightfield + normal
ACTIVE_PER_PASS = 36 + 9 * 15 + 21 * 6 + 18 * 6 + 6 * 6 + 6 * 6 + 3 * 6 + 11   # J^T W J, J^T f
ACTIVE_STATUS = CROSS + 3 + DOT3 + 4 + 6 + 7 + 8


def physics_flop_per_env_substep(num_candidates, active_contacts=4.0, heightfield=True):
    """FLOP of one env-substep of lgx_physics_kernel's algorithm.

    num_candidates: contact primitives of the robot model (Go1 92, ANYmal-C 37);
    active_contacts: primitives in contact (nominal stance: 4 feet)."""
    legs = 4
    free = (QUAT_TO_MAT + 12 * KIN_PER_JOINT + 13 * BODY_SI + 12 * RNEA_PER_JOINT + legs * RNEA_LEG_SUMS + FBASE
            + legs * CRBA_PER_LEG + ACOM + RBCOM + legs * (RB0_PER_LEG + RL0_PER_LEG) + 12 * DRIVE_PER_JOINT
            + 2 * (legs * ARROW_PER_LEG + ARROW_PER_ENV) + legs * STATUS_VL_PER_LEG + INTEGRATE)
    geo = CAND_TRANSFORM + (HEIGHT_FIELD if heightfield else HEIGHT_PLANE)
    cand = num_candidates * geo                       # pass 0 classifies every primitive
    act = active_contacts * (geo + 2 * ACTIVE_PER_PASS + ACTIVE_STATUS)   # pass 1 revisits contacts only
    return free + cand + act


def actuator_mlp_flop_per_row(dims=(30, 128, 128, 128, 3)):
    return 2 * sum(a * b for a, b in zip(dims[:-1], dims[1:]))


def _macs(dims):
    return sum(a * b for a, b in zip(dims[:-1], dims[1:]))


def policy_flop_per_sample(actor_dims, critic_dims):
    """(rollout forward, one PPO epoch) FLOP per sample of the rsl_rl ActorCritic
    (SURVEY.md §8 a15/a16): forward = both nets; an epoch = forward + weight gradients of every
    layer + input gradients of every layer but the first (the observations need none)."""
    fwd = _macs(actor_dims) + _macs(critic_dims)
    first = actor_dims[0] * actor_dims[1] + critic_dims[0] * critic_dims[1]
    return 2 * fwd, 2 * (fwd + fwd + (fwd - first))


if __name__ == "__main__":
    print("policy (235-obs) fwd / epoch FLOP per sample:",
          policy_flop_per_sample((235, 512, 256, 128, 12), (235, 512, 256, 128, 1)))
    for name, nc, hf in (("go1 plane", 92, False), ("go1 rough", 92, True), ("anymal_c rough", 37, True)):
        print(f"{name:16s} {physics_flop_per_env_substep(nc, 4.0, hf):8.0f} FLOP/env-substep")
