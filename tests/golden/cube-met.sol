MeshVersionFormatted 2

Dimension 3

SolAtVertices
12
1 1
0.5
0.5
0.5
0.5
0.5
0.5
0.5
0.5
0.5
0.5
0.5
0.5

End