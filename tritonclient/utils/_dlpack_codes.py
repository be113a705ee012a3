"""DLPack type codes (dlpack.h v1.x)."""
kDLInt = 0
kDLUInt = 1
kDLFloat = 2
kDLBfloat = 4
kDLBool = 6
kDLFloat8_e4m3fn = 10
kDLFloat8_e5m2 = 12
