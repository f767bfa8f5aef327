"""How often an observation column formed as x * RN(1/d) differs from the
reference's x / d after the float32 rounding of an observation row
(frame.h observe_values): every integer spawn position and 2e7 uniform
values per divisor.  Prints the counts; 0 expected."""
import numpy as np


def main(n=20_000_000):
    rng = np.random.default_rng(0)
    for d in (800.0, 600.0, 10.0, 180.0, 1000.0):
        inv = 1.0 / d
        ints = np.arange(-2000, 2001, dtype=np.float64)
        x = rng.uniform(-1000, 1000, n)
        bad_int = int(((ints * inv).astype(np.float32) != (ints / d).astype(np.float32)).sum())
        bad_rand = int(((x * inv).astype(np.float32) != (x / d).astype(np.float32)).sum())
        f64 = float((x * inv != x / d).mean())
        print(f"d={d:g}: float32 rows differ on {bad_int} of {ints.size} integers, {bad_rand} of {n} uniform "
              f"values (the doubles differ by an ulp on {f64:.1%})")


if __name__ == "__main__":
    main()
