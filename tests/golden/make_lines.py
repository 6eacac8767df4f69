"""Tiny synthetic text-line datasets in the reference's CSV format (data/dataset.py:23-156:
`filename,text` rows with a header, images under a root directory), rendered with DejaVu fonts.
Written by this script (no reference code involved); committed under tests/golden/lines/ for the
training.train tests (tests/test_train_api.py).

    python tests/golden/make_lines.py            # regenerates tests/golden/lines/
"""
import csv
import os
import random

from PIL import Image, ImageDraw, ImageFont

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "lines")
FONTS = ["/usr/share/fonts/truetype/dejavu/DejaVuSans.ttf", "/usr/share/fonts/truetype/dejavu/DejaVuSansMono.ttf",
         "/usr/share/fonts/truetype/dejavu/DejaVuSerif.ttf"]
ALPHABET = "abcdefghijklmnopqrstuvwxyz0123456789"


def words(rng, n_min=1, n_max=2):
    return " ".join("".join(rng.choice(ALPHABET) for _ in range(rng.randint(2, 6)))
                    for _ in range(rng.randint(n_min, n_max)))


def render(text, rng, height=32):
    """dark text on a light background, left margin jittered; mode L or RGB (both decoders)"""
    font = ImageFont.truetype(rng.choice(FONTS), size=rng.randint(18, 24))
    x0, y0, x1, y1 = font.getbbox(text)
    w = x1 + 8 + rng.randint(0, 6)
    img = Image.new("L", (w, height), color=rng.randint(215, 255))
    ImageDraw.Draw(img).text((4 + rng.randint(0, 3), (height - (y1 - y0)) // 2 - y0), text,
                             fill=rng.randint(0, 50), font=font)
    return img.convert("RGB") if rng.random() < 0.5 else img


def write_set(root, n, rng, header=True, prefix="img"):
    os.makedirs(root, exist_ok=True)
    rows = []
    for i in range(n):
        t = words(rng)
        fn = f"{prefix}_{i:03d}.png"
        render(t, rng).save(os.path.join(root, fn), optimize=True)
        rows.append((fn, t))
    with open(os.path.join(root, "labels.csv"), "w", newline="", encoding="utf-8") as f:
        w = csv.writer(f)
        if header:
            w.writerow(["filename", "text"])
        w.writerows(rows)


def main():
    rng = random.Random(20261017)
    write_set(os.path.join(OUT, "a"), 40, rng)                     # split by val_size
    write_set(os.path.join(OUT, "b", "train"), 24, rng, header=False, prefix="tr")
    write_set(os.path.join(OUT, "b", "val"), 8, rng, prefix="va")   # a separate val set


if __name__ == "__main__":
    main()
