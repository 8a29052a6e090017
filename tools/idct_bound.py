# Interval bound behind the 32-bit product test of idct_block (ffcv_amd/csrc/ffcv_jpeg.hip, fmul8).
# interval bound of jidctfst ifast (jpeg_idct_ifast) products, inputs |d| <= 1
def mul(v, c): return v * abs(c) / 256.0
def col(d):  # d: list of 8 bounds (rows 0..7 of one column)
    t0,t1,t2,t3 = d[0],d[2],d[4],d[6]
    m = []
    t10=t0+t2; t11=t0+t2; t13=t1+t3
    m.append(t1+t3)             # (tmp1 - tmp3) * 362
    t12=mul(t1+t3,362)+t13
    a0=t10+t13; a3=t10+t13; a1=t11+t12; a2=t11+t12
    t4,t5,t6,t7 = d[1],d[3],d[5],d[7]
    z13=t6+t5; z10=t6+t5; z11=t4+t7; z12=t4+t7
    T7=z11+z13
    m += [z11+z13, z10+z12, z12, z10]   # *362, *473, *277, *669
    T11=mul(z11+z13,362); z5=mul(z10+z12,473); T10=mul(z12,277)+z5; T12=mul(z10,669)+z5
    T6=T12+T7; T5=T11+T6; T4=T10+T5
    out=[a0+T7, a1+T6, a2+T5, a3+T4, a3+T4, a2+T5, a1+T6, a0+T7]
    consts=[362,362,473,277,669]
    prods=[mi*c for mi,c in zip(m,consts)]
    return out, max(prods)
p1, m1 = col([1.0]*8)
P = max(p1)
p2, m2 = col([P]*8)
print('pass-1 output bound', P, 'max product pass1', m1, 'pass2', m2)
print('max |d| for exact 32-bit products: < %.1f' % ((2**31 - 1) / max(m1, m2)))
