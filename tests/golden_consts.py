"""Constants shared by the golden fixtures (examples/example.par:4,8)."""
P0 = 1.0 / 345.67890123456789
DM0 = 34.56789
