"""CPU: the rendering oracle (oracle/render.py) and the glyph atlas it shares
with dd_render, checked against the facts the reference's render code fixes
(colours, rectangles, text positions: game_engine.py:300-412,
platform.py:76-102, drone.py:155-218).  pygame itself is absent, so pixel
parity with pygame is unpinned."""
import numpy as np

from oracle import render as R

BASE = dict(x=200.0, y=300.0, vx=0.0, vy=0.0, angle=0.0, fuel=1000.0, px=600.0, py=450.0,
            total_reward=0.0, status=0, steps=3, episode=1)


def lane(**kw):
    d = dict(BASE)
    d.update(kw)
    return d


def test_atlas_faces_cover_every_string_the_reference_draws():
    height, index, offset, advance, cov = R.atlas()
    assert list(height) == [19, 24, 39]
    for ch in "Fuel: Speed Angle Distance Episode Steps Total Reward Press R to restart 0123456789.-":
        assert index[ord(ch)] >= 0, ch
    assert index[R.DEGREE] >= 0
    assert index[128 + ord("H")] >= 0
    for ch in "SUCCESSFUL LANDING! CRASHED!":
        assert index[256 + ord(ch)] >= 0, ch
    assert int(offset[-1] + height[2] * advance[-1]) == len(cov)
    assert cov.max() == 255


def test_scene_colours_and_rectangles():
    img = R.render(lane(), hud=False)
    assert img.shape == (600, 800, 3) and img.dtype == np.uint8
    assert tuple(img[100, 400]) == R.SKY
    assert tuple(img[550, 0]) == R.GROUND and tuple(img[549, 0]) == R.SKY   # ground rect at y = 550
    # platform (550, 440, 100, 20): 2-px outline, fill, centre line at x = 600, 601, rows 440..460
    assert tuple(img[440, 550]) == R.OUTLINE and tuple(img[441, 551]) == R.OUTLINE
    assert tuple(img[442, 552]) == R.PLATFORM
    assert tuple(img[459, 649]) == R.OUTLINE and tuple(img[460, 560]) == R.SKY
    assert tuple(img[441, 600]) == R.WHITE and tuple(img[441, 601]) == R.WHITE
    assert tuple(img[460, 600]) == R.WHITE   # the line's end point (py + 10) is drawn
    assert tuple(img[442, 599]) == R.PLATFORM


def test_upright_drone_sprite():
    img = R.render(lane(), hud=False)
    # 40 x 20 sprite centred on (200, 300): columns 180..219, rows 290..309
    assert tuple(img[300, 200]) == R.HUB
    assert tuple(img[300, 185]) == R.ROTOR and tuple(img[300, 215]) == R.ROTOR
    assert tuple(img[291, 195]) == R.DRONE
    assert tuple(img[289, 200]) == R.SKY and tuple(img[310, 200]) == R.SKY
    assert tuple(img[300, 179]) == R.SKY and tuple(img[300, 220]) == R.SKY


def test_rotation_and_flames_follow_rotate_point():
    img = R.render(lane(angle=90.0), action=7, hud=False)
    # rotated a quarter turn clockwise: the sprite now spans rows 280..319, columns 190..209
    assert tuple(img[281, 200]) != R.SKY and tuple(img[318, 200]) != R.SKY
    assert tuple(img[285, 185]) == R.SKY
    # main flame: rotate_point(0, 17.5, 90) = (-17.5, 0) -> centre (182, 300), ellipse 16 x 15
    assert tuple(img[300, 182]) == R.THRUST and tuple(img[300, 175]) == R.THRUST
    # side flames at rotate_point(-/+25, 0, 90) = (0, -/+25): (200, 275), (200, 325)
    assert tuple(img[275, 200]) == R.THRUST and tuple(img[325, 200]) == R.THRUST
    none = R.render(lane(angle=90.0, fuel=0.0), action=7, hud=False)  # no flames without fuel
    assert tuple(none[275, 200]) == R.SKY and tuple(none[300, 178]) == R.SKY


def test_hud_fuel_bar_colours():
    for fuel, col in ((1000.0, R.GREEN), (250.0, R.YELLOW), (50.0, R.RED)):
        img = R.render(lane(fuel=fuel))
        assert tuple(img[28, 11]) == col, fuel
        assert tuple(img[28, 209]) == (R.BAR_BG if fuel < 1000 else R.GREEN)


def test_game_over_overlay_halves_and_titles():
    img = R.render(lane(status=1 | 4), hud=False)
    assert tuple(img[100, 50]) == tuple(c // 2 for c in R.SKY)
    title = img[255:290, 300:500].reshape(-1, 3)
    assert (title == np.array(R.RED)).all(axis=1).any()
    img = R.render(lane(status=1 | 2), hud=False)
    title = img[255:290, 200:600].reshape(-1, 3)
    assert (title == np.array(R.GREEN)).all(axis=1).any()


def test_text_layout_is_the_sum_of_advances():
    _, index, _, advance, _ = R.atlas()
    m = R.text_mask("Fuel: 250", 0)
    assert m.shape == (19, sum(int(advance[index[ord(c)]]) for c in "Fuel: 250"))
