"""Unit system of sclmd (sclmd/units.py:5-10): hbar = 1, energies in eV, time unit
0.658211814201041 fs, mass-weighted lengths in units of 0.06466 Angstrom*sqrt(amu)."""
time = 0.658211814201041e-15   # seconds per time unit
ohbar = 0.06466                # length scaling that makes hbar = 1
hbar = 1.0
kb = 0.000086173423            # eV / K
length = ohbar
curcof = 243414.0              # eV per time unit -> nW (heat current)

# Atomic masses (amu) keyed by element label, including sclmd's coarse-grained C1-C4 and Au1-Au4
# pseudo-atoms (units.py:16-46).  Stored as text and parsed once.
_MASSES = """
H 1.00794 He 4.002602 Li 6.941 Be 9.012182 B 10.811 C 12.0107 N 14.0067 O 15.9994 F 18.9984032
Ne 20.1791 Na 22.98976928 Mg 24.3050 Al 26.9815386 Si 28.0855 P 30.973762 S 32.065 Cl 35.453
Ar 39.948 K 39.0983 Ca 40.078 Sc 44.955912 Ti 47.867 V 50.9415 Cr 51.9961 Mn 54.938045 Fe 55.845
Co 58.933195 Ni 58.6934 Cu 63.546 Zn 65.38 Ga 69.723 Ge 72.64 As 74.92160 Se 78.96 Br 79.904
Kr 83.798 Rb 85.4678 Sr 87.62 Y 88.90585 Zr 91.224 Nb 92.90638 Mo 95.96 Tc 98 Ru 101.07
Rh 102.90550 Pd 106.42 Ag 107.8682 Cd 112.411 In 114.818 Sn 118.710 Sb 121.760 Te 127.60
I 126.90447 Xe 131.293 Cs 132.9054519 Ba 137.327 La 138.90547 Ce 140.116 Pr 140.90765 Nd 144.242
Pm 145 Sm 150.36 Eu 151.964 Gd 157.25 Tb 158.92535 Dy 162.500 Ho 164.93032 Er 167.259
Tm 168.93421 Yb 173.054 Lu 174.9668 Hf 178.49 Ta 180.94788 W 183.84 Re 186.207 Os 190.23
Ir 192.217 Pt 195.084 Au 196.966569 Hg 200.59 Tl 204.3833 Pb 207.2 Bi 208.98040 Po 209 At 210
Rn 222 Fr 223 Ra 226 Ac 227 Th 232.03806 Pa 231.03586 U 238.02891 Np 237 Pu 244 Am 243 Cm 247
Bk 247 Cf 251 Es 252 Fm 257 Md 258 No 259 Lr 262 Rf 265 Db 268 Sg 271 Bh 272 Hs 270 Mt 276
Ds 281 Rg 280 Cn 285 Uut 284 Uuq 289 Uup 288 Uuh 293 Uus 294 Uuo 294
C1 24.0214 C2 48.0428 C3 96.0856 C4 192.1712
Au1 98.4832845 Au2 49.24164225 Au3 24.620821125 Au4 12.3104105625
"""
_tok = _MASSES.split()
AtomicMassTable = {_tok[i]: float(_tok[i + 1]) for i in range(0, len(_tok), 2)}
del _tok
