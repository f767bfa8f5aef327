#!/bin/bash
# Timing-only builds of the step kernel for A/B runs (tools/kernel_lab.py).
# Each is the product source with one -D switch; outputs go to _native/lab/.
set -e
cd "$(dirname "$0")/../reinforcement-learning-101_amd"
OUT=delivery_drone_amd/_native/lab
mkdir -p $OUT
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -I../include -Ibuild"
build() { /opt/rocm/bin/hipcc $FLAGS "${@:2}" -o $OUT/lib_$1.so csrc/drone_step.hip csrc/policy_mlp.hip csrc/policy_rollout.hip csrc/render.hip & }
# "prev": the committed source at $PREV_REV (default HEAD), for before/after runs
if [ -n "${PREV_REV:-HEAD}" ] && git -C .. rev-parse -q --verify "${PREV_REV:-HEAD}" > /dev/null 2>&1; then
  mkdir -p /tmp/dd_prev
  git -C .. show "${PREV_REV:-HEAD}:reinforcement-learning-101_amd/csrc/drone_step.hip" > /tmp/dd_prev/drone_step.hip
  PREV_SRCS=/tmp/dd_prev/drone_step.hip
  for f in trig.h philox.h frame.h libm_ref.h mlp_core.h policy_mlp.hip policy_rollout.hip render.hip font_atlas.h; do
    git -C .. show "${PREV_REV:-HEAD}:reinforcement-learning-101_amd/csrc/$f" > /tmp/dd_prev/$f 2>/dev/null || rm -f /tmp/dd_prev/$f
  done
  [ -f /tmp/dd_prev/policy_mlp.hip ] && PREV_SRCS="$PREV_SRCS /tmp/dd_prev/policy_mlp.hip"
  [ -f /tmp/dd_prev/policy_rollout.hip ] && PREV_SRCS="$PREV_SRCS /tmp/dd_prev/policy_rollout.hip"
  [ -f /tmp/dd_prev/render.hip ] && PREV_SRCS="$PREV_SRCS /tmp/dd_prev/render.hip"
  /opt/rocm/bin/hipcc $FLAGS -Icsrc -o $OUT/lib_prev.so $PREV_SRCS &
fi
for v in ${VARIANTS:-base}; do
  case $v in
    base) build base ;;
    flat) build flat -DDD_EXP_FLAT_NEAR ;;
    s0lds) build s0lds -DDD_EXP_S0_LDS ;;
    flats0) build flats0 -DDD_EXP_FLAT_NEAR -DDD_EXP_S0_LDS ;;
    sel) build sel -DDD_EXP_SEL ;;
    ocml) build ocml -DDD_TRIG_OCML ;;
    plainobs) build plainobs -DDD_ST_OBS=0 ;;
    nofma) build nofma -DDD_TRIG_NO_FMA ;;
    plainout) build plainout -DDD_ST_OUT=0 ;;
    nomath) build nomath -DDD_EXP_NOMATH ;;
    mlpw4) build mlpw4 -DDD_MLP_WAVES=4 ;;
    mlpw12) build mlpw12 -DDD_MLP_WAVES=12 ;;
    empty) build empty -DDD_EXP_EMPTY ;;
    b512) build b512 -DDD_STEP_BLOCK=512 ;;
    b1024) build b1024 -DDD_STEP_BLOCK=1024 ;;
    b128) build b128 -DDD_STEP_BLOCK=128 ;;
    w8) build w8 -DDD_STEP_MIN_WAVES=8 ;;
    w4) build w4 -DDD_STEP_MIN_WAVES=4 ;;
    rw2) build rw2 -DDD_ROLL_MIN_WAVES=2 ;;
    rw4) build rw4 -DDD_ROLL_MIN_WAVES=4 ;;
    lateact) build lateact -DDD_EXP_LATE_ACT ;;
    wrapsel) build wrapsel -DDD_EXP_STEP_WRAP_SELECT ;;
    wts) build wts -DDD_ST_STATE=1 ;;
    wto) build wto -DDD_ST_OUT=1 -DDD_ST_OBS=1 ;;
    wtall) build wtall -DDD_ST_STATE=1 -DDD_ST_OUT=1 -DDD_ST_OBS=1 ;;
    wtntall) build wtntall -DDD_ST_STATE=3 -DDD_ST_OUT=3 -DDD_ST_OBS=3 ;;
    wtsnto) build wtsnto -DDD_ST_STATE=1 -DDD_ST_OUT=3 -DDD_ST_OBS=3 ;;
    plainall) build plainall -DDD_ST_OUT=0 -DDD_ST_OBS=0 ;;
    faketrig) build faketrig -DDD_EXP_FAKE_TRIG ;;
    fakesqrt) build fakesqrt -DDD_EXP_FAKE_SQRT ;;
    emptyb1024) build emptyb1024 -DDD_EXP_EMPTY -DDD_STEP_BLOCK=1024 ;;
    tl) build tl -DDD_EXP_TIMELINE ;;
    tlnomath) build tlnomath -DDD_EXP_TIMELINE -DDD_EXP_NOMATH ;;
    tlwtsnto) build tlwtsnto -DDD_EXP_TIMELINE -DDD_ST_STATE=1 -DDD_ST_OUT=3 -DDD_ST_OBS=3 ;;
    tlwtall) build tlwtall -DDD_EXP_TIMELINE -DDD_ST_STATE=1 -DDD_ST_OUT=1 -DDD_ST_OBS=1 ;;
    ieeerstd) build ieeerstd -DDD_MLP_IEEE_RSTD ;;
    sl*) build $v -DDD_EXP_STEP_DYN_LDS=${v#sl} ;;
    rl*) build $v -DDD_EXP_ROLL_DYN_LDS=${v#rl} ;;
    pad*) build $v -DDD_EXP_PAD_VALU=${v#pad} ;;
    glibctrig) build glibctrig -DDD_TRIG_GLIBC ;;
    noexact) build noexact -DDD_EXP_NO_EXACT ;;
    sqrtllvm) build sqrtllvm -DDD_SQRT_LLVM ;;
    vcoef) build vcoef -DDD_EXP_TRIG_VCOEF ;;
    fakespawn) build fakespawn -DDD_EXP_FAKE_SPAWN ;;
    nolicm) build nolicm -mllvm -disable-machine-licm ;;
    count) build count -DDD_EXP_COUNT ;;
    exactcall) build exactcall -DDD_EXP_EXACT_CALL ;;
    exactlds) build exactlds -DDD_EXP_EXACT_LDS ;;
    riskyonly) build riskyonly -DDD_EXP_RISKY_ONLY ;;
    defer) build defer -DDD_EXP_DEFER_REDO ;;
    maxilp) build maxilp -mllvm -amdgpu-sched-strategy=max-ilp ;;
    iterilp) build iterilp -mllvm -amdgpu-sched-strategy=iterative-ilp ;;
    itermin) build itermin -mllvm -amdgpu-sched-strategy=iterative-minreg ;;
    mpad*) build $v -DDD_MLP_PAD=${v#mpad} ;;
    ref*) build $v -DDD_SPAWN_REFILL=${v#ref} ;;
    log1p) build log1p -DDD_MLP_LOG1P ;;
    serial) build serial -DDD_MLP_SERIAL ;;
    splitcvt) build splitcvt -DDD_MLP_SPLIT_CVT ;;
    uncentered) build uncentered -DDD_MLP_UNCENTERED ;;
    tl_s*_o*)  # timeline + store policies: tl_s<state>_o<out and obs>, values as DD_ST_* (>= 100: raw aux bits)
      s=${v#tl_s}; s=${s%%_o*}; o=${v##*_o}
      build $v -DDD_EXP_TIMELINE -DDD_ST_STATE=$s -DDD_ST_OUT=$o -DDD_ST_OBS=$o ;;
    *) echo "unknown variant $v" >&2; exit 1 ;;
  esac
done
wait
ls -la $OUT
